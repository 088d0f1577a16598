"""Keras `.h5` weight files for cFlow, without TensorFlow or h5py.

The reference checkpoints with `model.save_weights(path.h5)` and restores with
`model.load_weights(path)` (conv_cINN.py:579,641; conv_pre_training_cINN_on_noise.py:138,147;
ModelCheckpoint(save_weights_only=True) conv_cINN.py:522-526). TF 2.7's Keras (the version the
reference's README names) writes such a file as

* root attributes `layer_names` (every entry of `model.layers`, fixed-length byte strings),
  `backend` = b'tensorflow', `keras_version`;
* one group per layer, attribute `weight_names` (the layer's `trainable + non_trainable`
  variable names), one dataset per variable at `<group>/<variable name>`, e.g.
  `coupling_layer_2/conv2d_17/kernel:0`;

and `load_weights` assigns BY ORDER: the i-th layer-with-weights of the file to the i-th of
the model, the j-th name in `weight_names` to the j-th variable (shapes checked).

How that order maps onto this package's canonical parameter order (make_model.param_specs,
oracle/cflow_np.py:param_specs):

* `model.layers` of cFlow = `layers_list` (coupling / squeeze / factor layers in flow order,
  conv_cINN_make_model.py:1630-1689) followed by the four `Mean` loss trackers
  (:1692-1695), which carry weights `total:0` / `count:0`; squeeze and factor layers have none;
* a coupling layer's variables = model_A's then model_b's (`self.model_A, self.model_b =
  self.coupling_function()`, :439; children gathered in tracking order), and a functional
  model's variables follow its layers by decreasing depth, which for these chain-shaped nets is
  forward order: conv_in, per residual block LN1, conv_a, LN2, the grouped branches (dilation-
  major, group-minor), LN3, conv_b, then LN_out, conv_out, tanh scale — exactly the canonical
  order within a coupling;
* variable names come from Keras's per-class layer counters in creation order:
  coupling_function builds net b before net A (:1120-1206), so within a coupling the b-net convs
  take the lower `conv2d_N` numbers.

The HDF5 container is pinned against h5py 3.3 / libhdf5 (tests/test_h5weights.py). The
Keras-side facts above (model.layers membership of the metric trackers, variable naming) are
read from the Keras 2.7 sources' behaviour, not observed: TensorFlow is absent here, so the
name / order mapping is "parity unpinned". The importer therefore keys only on what Keras's own
loader keys on — layer order, weight order and shapes — and skips groups whose variables are
only metric state (`total`, `count`), so a file with or without the trackers loads.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import h5lite

KERAS_VERSION = '2.7.0'
METRIC_NAMES = ('loss', 'z_loss', 'y_loss', 'detJ_loss')   # conv_cINN_make_model.py:1692-1695


def _coupling_groups(specs: Sequence[Tuple[str, tuple]]) -> List[List[Tuple[str, tuple]]]:
    """Canonical specs split per coupling layer (names 'c<idx>.<A|b>.…'), in order."""
    groups: List[List[Tuple[str, tuple]]] = []
    cur = None
    for name, shape in specs:
        key = name.split('.', 1)[0]
        if key != cur:
            groups.append([])
            cur = key
        groups[-1].append((name, tuple(shape)))
    return groups


def _kind(name: str) -> str:
    """Keras layer class of a canonical parameter: conv2d / layer_normalization / tanh."""
    part = name.split('.')[-2]
    if part.startswith('ln'):
        return 'layer_normalization'
    if part == 'tanh_scale':
        return 'tanh_scaling_layer'
    return 'conv2d'


def _var(name: str) -> str:
    leaf = name.split('.')[-1]
    return {'kernel': 'kernel', 'bias': 'bias', 'gamma': 'gamma', 'beta': 'beta', 'w': 'Variable'}[leaf]


def _uniq(prefix: str, n: int) -> str:
    return prefix if n == 0 else f'{prefix}_{n}'


def keras_names(layer_kinds: Sequence[str], specs: Sequence[Tuple[str, tuple]]):
    """-> (layer names of model.layers, {layer name: [(weight name, canonical name)]}) as a fresh
    TF 2.7 session would name a cFlow built with this architecture."""
    counters: Dict[str, int] = {}

    def take(prefix):
        n = counters.get(prefix, 0)
        counters[prefix] = n + 1
        return _uniq(prefix, n)

    cgroups = _coupling_groups(specs)
    layer_names: List[str] = []
    weights: Dict[str, List[Tuple[str, str]]] = {}
    ci = 0
    cls = {'coupling': 'coupling_layer', 'squeeze': 'squeeze_layer', 'factor': 'factor_out_zy_layer'}
    for kind in layer_kinds:
        lname = take(cls[kind])
        layer_names.append(lname)
        if kind != 'coupling':
            weights[lname] = []
            continue
        group = cgroups[ci]
        ci += 1
        # Keras layer instances of this coupling: consecutive canonical params of one class and
        # one canonical layer prefix form one Keras layer
        insts: Dict[str, List[str]] = {}   # canonical layer prefix -> params
        order: List[str] = []
        for name, _ in group:
            pre = name.rsplit('.', 1)[0]
            if pre not in insts:
                insts[pre] = []
                order.append(pre)
            insts[pre].append(name)
        # creation order: net b's layers, then net A's (coupling_function :1120-1206)
        created = [p for p in order if p.split('.')[1] == 'b'] + [p for p in order if p.split('.')[1] == 'A']
        kname = {p: take(_kind(insts[p][0])) for p in created}
        weights[lname] = [(f'{kname[p]}/{_var(n)}:0', n) for p in order for n in insts[p]]
    if ci != len(cgroups):
        raise ValueError(f'{len(cgroups)} coupling parameter groups for {ci} coupling layers')
    for m in METRIC_NAMES:
        layer_names.append(m)
        weights[m] = [('total:0', None), ('count:0', None)]
    return layer_names, weights


def save_h5(path, layer_kinds, specs, values: Dict[str, np.ndarray]) -> None:
    """Write a Keras-layout weight file (keras hdf5_format.save_weights_to_hdf5_group)."""
    layer_names, weights = keras_names(layer_kinds, specs)
    shapes = dict((n, tuple(s)) for n, s in specs)
    w = h5lite.Writer()
    w.attrs['layer_names'] = np.array([n.encode('utf-8') for n in layer_names])
    w.attrs['backend'] = b'tensorflow'
    w.attrs['keras_version'] = KERAS_VERSION.encode('utf-8')
    for lname in sorted(layer_names):
        g = w.create_group(lname)
        wl = weights[lname]
        g.attrs['weight_names'] = np.array([k.encode('utf-8') for k, _ in wl]) if wl else np.zeros(0, np.float64)
        for kname, cname in wl:
            if cname is None:
                val = np.float32(0)   # fresh tracker state
            else:
                val = np.asarray(values[cname], dtype=np.float32).reshape(shapes[cname])
            g.create_dataset(kname, val)
    w.save(path)


def _str_list(v) -> List[str]:
    a = np.asarray(v).reshape(-1)
    return [x.decode('utf-8') if isinstance(x, (bytes, np.bytes_)) else str(x) for x in a]


def _attr_list(group, name) -> List[str]:
    """keras hdf5_format.load_attributes_from_hdf5_group: `name` or chunks `name0`, `name1`, …"""
    if name in group.attrs:
        return _str_list(group.attrs[name]) if np.asarray(group.attrs[name]).size else []
    out, k = [], 0
    while f'{name}{k}' in group.attrs:
        out.extend(_str_list(group.attrs[f'{name}{k}']))
        k += 1
    return out


def load_h5(path, layer_kinds, specs) -> Dict[str, np.ndarray]:
    """Read a Keras weight file into {canonical name: array}, assigning by order as keras
    hdf5_format.load_weights_from_hdf5_group does; raises ValueError on count / shape mismatch."""
    f = h5lite.File(path)
    if 'layer_names' not in f.attrs and 'layer_names0' not in f.attrs:
        raise ValueError(f'{path}: not a Keras weight file (no layer_names attribute)')
    filtered = []
    for lname in _attr_list(f, 'layer_names'):
        g = f[lname]
        names = _attr_list(g, 'weight_names')
        if not names:
            continue
        if all(n.split('/')[-1].split(':')[0] in ('total', 'count') for n in names):
            continue   # metric tracker state: not part of the flow
        filtered.append((lname, g, names))
    cgroups = _coupling_groups(specs)
    n_coupling = sum(1 for k in layer_kinds if k == 'coupling')
    if len(filtered) != n_coupling or len(cgroups) != n_coupling:
        raise ValueError(f'You are trying to load a weight file containing {len(filtered)} layers into a model '
                         f'with {n_coupling} layers.')
    out: Dict[str, np.ndarray] = {}
    for k, ((lname, g, names), group) in enumerate(zip(filtered, cgroups)):
        if len(names) != len(group):
            raise ValueError(f'Layer #{k} (named "{lname}") expects {len(group)} weight(s), but the saved weights '
                             f'have {len(names)} element(s).')
        for wname, (cname, shape) in zip(names, group):
            val = np.asarray(g[wname].read())
            if tuple(val.shape) != tuple(shape):
                raise ValueError(f'Layer #{k} (named "{lname}"), weight {wname}: shape {tuple(val.shape)} '
                                 f'does not match the model\'s {cname} {tuple(shape)}')
            out[cname] = val.astype(np.float32)
    return out


def model_layout(model):
    """(layer kinds, canonical (name, shape) specs) of a make_model.cFlow."""
    from .make_model import coupling_layer, squeeze_layer
    kinds = ['coupling' if isinstance(L, coupling_layer) else 'squeeze' if isinstance(L, squeeze_layer) else 'factor'
             for L in model.layers_list]
    return kinds, [(n, s) for n, _, s in model.param_specs]


def save_weights_h5(model, path) -> None:
    kinds, specs = model_layout(model)
    save_h5(path, kinds, specs, model.get_weights())


def load_weights_h5(model, path) -> None:
    kinds, specs = model_layout(model)
    model.set_weights(load_h5(path, kinds, specs))
