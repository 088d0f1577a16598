"""Keras .h5 weight files: h5lite's HDF5 reader / writer and the Keras
layout mapping of keras_h5.py.

Pinning: tests/golden/keras_tiny.h5 was written by the real h5py 3.3 / libhdf5
(tests/golden/make_h5_golden.py, which follows TF 2.7 Keras's save_weights_to_hdf5_group), so
reading it exercises libhdf5's own encoding (vlen-string attributes in a global heap, symbol-
table groups, contiguous datasets). This writer's output is checked against the same fixture
with libhdf5's `h5diff -c` and read back by h5py, when the image's /opt/conda tools are present.
The Keras-side naming / order rules cannot be observed without TensorFlow (parity unpinned);
the fixture script states them independently of keras_h5.py.
"""
import os
import subprocess

import numpy as np
import pytest

from arl_conditional_normalizing_flows_amd import h5lite, keras_h5
from arl_conditional_normalizing_flows_amd.config import PRESETS
from oracle.cflow_np import OracleCFlow

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden', 'keras_tiny.h5')
CONDA_PY = '/opt/conda/bin/python3.9'
H5DIFF = '/opt/conda/bin/h5diff'


def _layout(name='tiny'):
    ora = OracleCFlow(**PRESETS[name].kwargs())
    return ora, [e.kind for e in ora.layers], ora.specs


def _params(ora, seed=1):
    return {k: np.asarray(v, np.float32) for k, v in ora.init_params(seed).items()}


def _conda_h5py():
    if not os.path.exists(CONDA_PY):
        return False
    r = subprocess.run([CONDA_PY, '-c', 'import h5py'], capture_output=True, timeout=60)
    return r.returncode == 0


def test_reads_h5py_written_keras_file():
    ora, kinds, specs = _layout()
    got = keras_h5.load_h5(GOLDEN, kinds, specs)
    P = _params(ora)
    assert set(got) == {n for n, _ in specs}
    for n, _ in specs:
        np.testing.assert_array_equal(got[n], P[n], err_msg=n)


def test_golden_layout_matches_keras_names():
    _, kinds, specs = _layout()
    f = h5lite.File(GOLDEN)
    layer_names, weights = keras_h5.keras_names(kinds, specs)
    assert [str(x) for x in f.attrs['layer_names']] == layer_names
    assert f.attrs['backend'] == 'tensorflow' and f.attrs['keras_version'] == keras_h5.KERAS_VERSION
    for ln in layer_names:
        assert keras_h5._attr_list(f[ln], 'weight_names') == [w for w, _ in weights[ln]], ln
    # the squeeze / factor groups hold an empty float64 attribute (np.asarray([])), like Keras
    assert np.asarray(f['squeeze_layer'].attrs['weight_names']).size == 0


def test_writer_roundtrip_and_sizes(tmp_path):
    ora, kinds, specs = _layout('small')
    P = _params(ora, seed=3)
    path = tmp_path / 'w.h5'
    keras_h5.save_h5(path, kinds, specs, P)
    got = keras_h5.load_h5(path, kinds, specs)
    for n, _ in specs:
        np.testing.assert_array_equal(got[n], P[n], err_msg=n)


@pytest.mark.skipif(not os.path.exists(H5DIFF), reason='libhdf5 h5diff not in this image')
def test_writer_equivalent_to_libhdf5_file(tmp_path):
    """h5diff -c (libhdf5) finds no difference in objects, data or attributes."""
    ora, kinds, specs = _layout()
    path = tmp_path / 'mine.h5'
    keras_h5.save_h5(path, kinds, specs, _params(ora))
    r = subprocess.run([H5DIFF, '-c', GOLDEN, str(path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.skipif(not _conda_h5py(), reason='no h5py interpreter in this image')
def test_h5py_reads_writer_output(tmp_path):
    w = h5lite.Writer()
    w.attrs['names'] = np.array([b'a', b'bcd'])
    w.attrs['count'] = np.int64(7)
    w.attrs['empty'] = np.zeros(0, np.float64)
    g = w.create_group('g/h')
    g.create_dataset('x:0', np.arange(24, dtype=np.float32).reshape(2, 3, 4))
    g.create_dataset('s', np.float32(2.5))
    w.create_dataset('d', np.linspace(0, 1, 5))
    for i in range(300):   # > 2*16 symbol nodes: two-level group B-tree
        w.create_dataset(f'many/e{i:03d}', np.full(3, i, np.int32))
    path = tmp_path / 'h.h5'
    w.save(path)
    script = (
        'import h5py, numpy as np, sys\n'
        'f = h5py.File(sys.argv[1], "r")\n'
        'names = [x.decode() if isinstance(x, bytes) else x for x in f.attrs["names"]]\n'
        'assert names == ["a", "bcd"], names\n'
        'assert int(f.attrs["count"]) == 7 and f.attrs["empty"].size == 0\n'
        'assert np.array_equal(f["g/h/x:0"][...], np.arange(24, dtype=np.float32).reshape(2, 3, 4))\n'
        'assert f["g/h/s"].shape == () and float(f["g/h/s"][()]) == 2.5\n'
        'assert np.allclose(f["d"][...], np.linspace(0, 1, 5))\n'
        'assert len(f["many"]) == 300 and all(int(f["many/e%03d" % i][1]) == i for i in range(300))\n'
        'print("ok")\n')
    r = subprocess.run([CONDA_PY, '-c', script, str(path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == 'ok', r.stdout + r.stderr


def test_h5lite_own_roundtrip_many_entries(tmp_path):
    w = h5lite.Writer()
    for i in range(600):
        w.create_dataset(f'grp/d{i:04d}', np.full(2, i, np.float64))
    w.create_dataset('scalar', np.float32(1.25))
    w.attrs['label'] = b'xyz'
    f = h5lite.File(w.save())
    assert f['grp'].keys() == [f'd{i:04d}' for i in range(600)]
    assert all(f[f'grp/d{i:04d}'].read()[0] == i for i in (0, 257, 599))
    s = f['scalar'].read()
    assert s.shape == () and s == np.float32(1.25)
    assert f.attrs['label'] == 'xyz'
    assert len(f.visit_datasets()) == 601


def test_load_rejects_wrong_architecture():
    _, kinds, specs = _layout('small')
    with pytest.raises(ValueError, match='layers|expects|shape'):
        keras_h5.load_h5(GOLDEN, kinds, specs)


def test_load_rejects_shape_mismatch(tmp_path):
    ora, kinds, specs = _layout()
    P = _params(ora)
    name = next(n for n, s in specs if n.endswith('conv_in.kernel'))
    bad = [(n, (s[0], s[1], s[2], s[3] + 1) if n == name else s) for n, s in specs]
    P[name] = np.zeros(dict(bad)[name], np.float32)
    path = tmp_path / 'bad.h5'
    keras_h5.save_h5(path, kinds, bad, P)
    with pytest.raises(ValueError, match='shape'):
        keras_h5.load_h5(path, kinds, specs)


def test_reader_rejects_non_hdf5(tmp_path):
    p = tmp_path / 'x.h5'
    p.write_bytes(b'not an hdf5 file' * 10)
    with pytest.raises(h5lite.H5Error):
        h5lite.File(p)
    data = open(GOLDEN, 'rb').read()
    with pytest.raises(h5lite.H5Error):
        keras_h5.load_h5(data[:2048], *_layout()[1:])


def test_file_without_metric_groups_loads(tmp_path):
    """Older / other Keras versions may not list the loss trackers in model.layers."""
    ora, kinds, specs = _layout()
    P = _params(ora, seed=5)
    layer_names, weights = keras_h5.keras_names(kinds, specs)
    w = h5lite.Writer()
    keep = [n for n in layer_names if n not in keras_h5.METRIC_NAMES]
    w.attrs['layer_names'] = np.array([n.encode() for n in keep])
    for ln in keep:
        g = w.create_group(ln)
        wl = weights[ln]
        g.attrs['weight_names'] = np.array([k.encode() for k, _ in wl]) if wl else np.zeros(0)
        for k, cname in wl:
            g.create_dataset(k, P[cname])
    got = keras_h5.load_h5(w.save(), kinds, specs)
    for n, _ in specs:
        np.testing.assert_array_equal(got[n], P[n])


@pytest.mark.gpu
def test_gpu_flow_from_keras_file_matches_oracle(gpu, tmp_path):
    """Load the h5py-written file into the HIP cFlow; its forward equals the oracle's on the same
    weights; save_weights(.h5) -> load_weights round-trips through the model."""
    import torch
    from arl_conditional_normalizing_flows_amd import training
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    from oracle.cflow_np import synthetic_class_batch
    cfg = PRESETS['tiny']
    flow = cFlow(**cfg.kwargs())
    training.load_weights(flow, GOLDEN)
    ora = OracleCFlow(**cfg.kwargs())
    P = _params(ora)
    for n, v in flow.get_weights().items():
        np.testing.assert_array_equal(v, P[n])
    H, W, _ = cfg.io_shape
    xy = synthetic_class_batch(2, H, W, cfg.x_d, seed=11)
    zy_ref, ld_ref = ora.forward(xy, P)
    zy, ld = flow(torch.from_numpy(xy).to(gpu), 1, per_image_logdet=True)
    torch.cuda.synchronize()
    e = float(np.max(np.abs(zy.cpu().numpy() - zy_ref)) / np.max(np.abs(zy_ref)))
    assert e < 1e-5
    assert np.max(np.abs(ld.cpu().numpy() - ld_ref)) <= 1e-4 * max(np.abs(ld_ref).max(), 1.0)
    out = tmp_path / 'saved.h5'
    training.save_weights(flow, out)
    flow2 = cFlow(**cfg.kwargs(), seed=9)
    training.load_weights(flow2, out)
    for n, v in flow2.get_weights().items():
        np.testing.assert_array_equal(v, P[n])
