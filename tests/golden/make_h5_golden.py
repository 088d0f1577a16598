#!/opt/conda/bin/python3.9
"""Write tests/golden/keras_tiny.h5 with the real h5py / libhdf5 (h5py 3.3 under the image's
/opt/conda/bin/python3.9; the package's own interpreter has no h5py).

The file follows what TF 2.7's Keras `model.save_weights('x.h5')` does for a cFlow
(keras/saving/hdf5_format.py save_weights_to_hdf5_group, as used by conv_cINN.py:641):
root attributes layer_names / backend / keras_version, one group per layer of model.layers
(sorted by name on creation), a `weight_names` attribute written through
save_attributes_to_hdf5_group (np.asarray of the byte strings; an empty list for layers
without weights), and `g.create_dataset(name, shape, dtype)` filled with `[:]` / `[()]`.
Layer / variable names follow Keras's per-class counters in creation order (net b before
net A inside coupling_function, conv_cINN_make_model.py:1120-1206); this script states that
rule independently of arl_conditional_normalizing_flows_amd/keras_h5.py.

The weights are the oracle's seeded fp32 initial parameters (oracle.cflow_np.init_params,
seed 1) for the 'tiny' preset; tests/test_h5weights.py regenerates them to compare.

    /opt/conda/bin/python3.9 tests/golden/make_h5_golden.py
"""
import os
import sys

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from oracle.cflow_np import OracleCFlow  # noqa: E402

SEED = 1


class Counter:
    def __init__(self):
        self.n = {}

    def __call__(self, prefix):
        k = self.n.get(prefix, 0)
        self.n[prefix] = k + 1
        return prefix if k == 0 else f'{prefix}_{k}'


def save_attributes_to_hdf5_group(group, name, data):
    data_npy = np.asarray(data)
    assert data_npy.nbytes < 64512   # no chunking needed at this size
    group.attrs[name] = data


def main():
    ora = OracleCFlow(**PRESETS['tiny'].kwargs())
    P = {k: np.asarray(v, np.float32) for k, v in ora.init_params(SEED).items()}
    uniq = Counter()
    layers = []   # (layer name, [(weight name, value)])
    ci = 0
    for e in ora.layers:
        if e.kind != 'coupling':
            layers.append((uniq('squeeze_layer' if e.kind == 'squeeze' else 'factor_out_zy_layer'), []))
            continue
        pre = f'c{e.coupling.index}'
        lname = uniq('coupling_layer')
        ci += 1
        names = [n for n, _ in ora.specs if n.startswith(pre + '.')]
        # Keras layers of this coupling, in canonical (= model.layers) order
        kl = []
        for n in names:
            lp = n.rsplit('.', 1)[0]
            if lp not in kl:
                kl.append(lp)
        kname = {}
        for net in ('b', 'A'):   # creation order
            for lp in kl:
                if lp.split('.')[1] != net:
                    continue
                tail = lp.split('.')[-1]
                cls = 'layer_normalization' if tail.startswith('ln') else \
                    'tanh_scaling_layer' if tail == 'tanh_scale' else 'conv2d'
                kname[lp] = uniq(cls)
        var = {'kernel': 'kernel:0', 'bias': 'bias:0', 'gamma': 'gamma:0', 'beta': 'beta:0', 'w': 'Variable:0'}
        ws = [(f'{kname[n.rsplit(".", 1)[0]]}/{var[n.rsplit(".", 1)[1]]}', P[n]) for n in names]
        layers.append((lname, ws))
    for m in ('loss', 'z_loss', 'y_loss', 'detJ_loss'):
        layers.append((m, [('total:0', np.float32(0)), ('count:0', np.float32(0))]))

    path = os.path.join(HERE, 'keras_tiny.h5')
    with h5py.File(path, 'w') as f:
        save_attributes_to_hdf5_group(f, 'layer_names', [n.encode('utf8') for n, _ in layers])
        f.attrs['backend'] = 'tensorflow'.encode('utf8')
        f.attrs['keras_version'] = '2.7.0'.encode('utf8')
        for lname, ws in sorted(layers, key=lambda x: x[0]):
            g = f.create_group(lname)
            save_attributes_to_hdf5_group(g, 'weight_names', [n.encode('utf8') for n, _ in ws])
            for n, val in ws:
                val = np.asarray(val)
                d = g.create_dataset(n.encode('utf8'), val.shape, dtype=val.dtype)
                if not val.shape:
                    d[()] = val
                else:
                    d[:] = val
    print(path, os.path.getsize(path), 'bytes,', ci, 'coupling layers')


if __name__ == '__main__':
    main()
