"""TFRecord / tf.train.Example restatement (create_tfrecords.py:150-238,
conv_cINN_base_functions.py:26-65). Pinned by: the CRC-32C check value of the standard
("123456789" -> 0xE3069283), protobuf's own runtime (google.protobuf, installed) decoding our
Example bytes through a descriptor built to tf.train.Example's schema, and round trips."""
import numpy as np
import pytest

from arl_conditional_normalizing_flows_amd import tfrecords as R


def test_crc32c_check_value():
    assert R.crc32c(b'123456789') == 0xE3069283          # RFC 3720 / iSCSI CRC-32C check value
    assert R.crc32c(b'') == 0


def _example_classes():
    """tf.train.Example's message schema, built with protobuf's descriptor API (no TF needed)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name='ex_test.proto', package='tfx', syntax='proto3')

    def msg(name, fields):
        m = fdp.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
        return m
    T = descriptor_pb2.FieldDescriptorProto
    msg('BytesList', [('value', 1, T.TYPE_BYTES, T.LABEL_REPEATED, None)])
    msg('FloatList', [('value', 1, T.TYPE_FLOAT, T.LABEL_REPEATED, None)])
    msg('Int64List', [('value', 1, T.TYPE_INT64, T.LABEL_REPEATED, None)])
    feat = msg('Feature', [('bytes_list', 1, T.TYPE_MESSAGE, T.LABEL_OPTIONAL, '.tfx.BytesList'),
                           ('float_list', 2, T.TYPE_MESSAGE, T.LABEL_OPTIONAL, '.tfx.FloatList'),
                           ('int64_list', 3, T.TYPE_MESSAGE, T.LABEL_OPTIONAL, '.tfx.Int64List')])
    feat.oneof_decl.add(name='kind')
    for f in feat.field:
        f.oneof_index = 0
    fs = msg('Features', [('feature', 1, T.TYPE_MESSAGE, T.LABEL_REPEATED, '.tfx.Features.FeatureEntry')])
    entry = fs.nested_type.add(name='FeatureEntry')
    entry.field.add(name='key', number=1, type=T.TYPE_STRING, label=T.LABEL_OPTIONAL)
    entry.field.add(name='value', number=2, type=T.TYPE_MESSAGE, label=T.LABEL_OPTIONAL, type_name='.tfx.Feature')
    entry.options.map_entry = True
    msg('Example', [('features', 1, T.TYPE_MESSAGE, T.LABEL_OPTIONAL, '.tfx.Features')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName('tfx.Example'))


def test_example_encoding_matches_protobuf_runtime():
    Example = _example_classes()
    img = np.random.default_rng(0).random((1, 4, 5, 2)).astype(np.float32)
    lab = np.eye(10, dtype=np.float32)[3:4]
    buf = R.encode_example({'img': img.tobytes(), 'height': 4, 'width': 5, 'depth': 2, 'label': lab.tobytes(),
                            'ints': [-3, 7], 'floats': np.array([1.5, -2.25], np.float32)})
    ex = Example()
    ex.ParseFromString(buf)
    f = ex.features.feature
    assert f['img'].bytes_list.value[0] == img.tobytes()
    assert list(f['height'].int64_list.value) == [4] and list(f['ints'].int64_list.value) == [-3, 7]
    assert list(f['floats'].float_list.value) == [1.5, -2.25]
    # and protobuf's serialisation decodes with ours
    back = R.decode_example(ex.SerializeToString())
    assert back['img'] == img.tobytes() and back['depth'] == [2] and back['ints'] == [-3, 7]
    assert np.array_equal(back['floats'], np.array([1.5, -2.25], np.float32))


def test_make_and_load_tfrecord_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    x = rng.random((5, 28, 28, 1)).astype(np.float32)
    y = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 5)]
    p = str(tmp_path / 'mnist.tfrecords')
    R.make_tfrecord(x, y, p)
    xi, yi = R.load_tfrecord(p)
    assert np.array_equal(xi, x) and np.array_equal(yi, y)
    # a flipped payload byte is caught by the record CRC
    raw = bytearray(open(p, 'rb').read())
    raw[40] ^= 1
    open(p, 'wb').write(bytes(raw))
    with pytest.raises(ValueError, match='CRC'):
        R.load_tfrecord(p)
