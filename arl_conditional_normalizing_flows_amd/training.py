"""Training driver: the reference's model.fit loop with its callbacks and
the annealed instance-noise schedule, over the HIP train_step / test_step.

  fit(...)                       keras Model.fit as conv_cINN.py:617-631 calls it (epochs,
                                 initial_epoch, validation_data, callbacks)
  EarlyStopping                  tf.keras.callbacks.EarlyStopping(monitor='val_loss', patience)
                                 (conv_cINN.py:140-141)
  CSVLogger                      tf.keras.callbacks.CSVLogger(path, separator=',', append=True)
                                 (:533-536): header 'epoch' + sorted metric names
  ModelCheckpoint                save_weights_only every save_freq batches, '{epoch:02d}' in the
                                 name (:522-527); weights as .npz (no h5py here)
  anneal_and_fit(...)            conv_cINN.py:583-636: num_annealing_epochs one-epoch fits on
                                 instance_noise(xy, alpha = i / num_annealing_epochs), then the
                                 clean fit up to num_epochs
  save_weights / load_weights    Keras-layout .h5 (keras_h5.py) or {canonical name: array} .npz
                                 (np.load with allow_pickle=False)

Datasets are iterables of device batches (torch tensors [B, H, W, D]); `callable` datasets are
re-invoked each epoch (the tf.data re-iteration of the reference).
"""
from __future__ import annotations

import csv
import math
import os
from typing import Callable, Iterable, List, Optional

import numpy as np

from .base_functions import instance_noise


def save_weights(model, path):
    """model.save_weights (conv_cINN.py:636-641). A path ending in .h5 / .hdf5 / .keras writes the
    Keras HDF5 layout the reference's files have (keras_h5.py); anything else a
    {canonical parameter name: array} .npz."""
    if str(path).endswith(('.h5', '.hdf5', '.keras')):
        from .keras_h5 import save_weights_h5
        save_weights_h5(model, path)
    else:
        # through an open handle: np.savez would append '.npz' to a bare path, and the file the
        # caller named (ModelCheckpoint.saved, load_weights) would not exist
        with open(path, 'wb') as fh:
            np.savez(fh, **model.get_weights())


def load_weights(model, path):
    """model.load_weights (conv_cINN.py:579): a Keras .h5 weight file (including one the
    reference wrote) or save_weights' .npz (no pickles)."""
    with open(path, 'rb') as fh:
        is_h5 = fh.read(8) == b'\x89HDF\r\n\x1a\n'
    if is_h5:
        from .keras_h5 import load_weights_h5
        load_weights_h5(model, path)
        return
    with np.load(path, allow_pickle=False) as z:
        model.set_weights({k: z[k] for k in z.files})


class Callback:
    """keras.callbacks.Callback subset. on_train_batch_end receives train_step's logs: 0-d float64
    DEVICE tensors (the running loss means, as TF's train_step returns tensors), so that the step
    needs no host read; float(v) there costs a device sync per batch. on_epoch_end receives host
    floats (the epoch's one read)."""
    # callbacks that write files run on rank 0 only in a data-parallel fit
    writes_files = False

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_train_batch_end(self, batch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass


class EarlyStopping(Callback):
    """monitor='val_loss', mode min, min_delta 0: stop once `patience` epochs pass without an
    improvement (keras semantics: wait resets on improvement; checked from the second epoch)."""

    def __init__(self, monitor='val_loss', patience=0, min_delta=0.0):
        self.monitor, self.patience, self.min_delta = monitor, int(patience), abs(float(min_delta))
        self.best, self.wait, self.stopped_epoch = math.inf, 0, None

    def on_train_begin(self, logs=None):
        self.best, self.wait, self.stopped_epoch = math.inf, 0, None

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        self.wait += 1
        if cur < self.best - self.min_delta:
            self.best, self.wait = cur, 0
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.model.stop_training = True


class CSVLogger(Callback):
    writes_files = True

    def __init__(self, filename, separator=',', append=False):
        self.filename, self.sep, self.append = filename, separator, append
        self.keys = None

    def on_train_begin(self, logs=None):
        self._has_header = self.append and os.path.exists(self.filename) and os.path.getsize(self.filename) > 0
        if not self.append:
            open(self.filename, 'w').close()

    def on_epoch_end(self, epoch, logs=None):
        logs = dict(logs or {})
        if self.keys is None:
            self.keys = sorted(logs)
        with open(self.filename, 'a', newline='') as f:
            w = csv.writer(f, delimiter=self.sep)
            if not self._has_header:
                w.writerow(['epoch'] + self.keys)
                self._has_header = True
            w.writerow([epoch] + [logs.get(k, 'NA') for k in self.keys])


class ModelCheckpoint(Callback):
    writes_files = True

    def __init__(self, filepath, save_weights_only=True, save_freq='epoch'):
        if not save_weights_only:
            raise NotImplementedError('only save_weights_only=True (the reference never saves whole models)')
        self.filepath, self.save_freq = filepath, save_freq
        self._batches, self._epoch = 0, 0
        self.saved: List[str] = []

    def _save(self, epoch):
        path = self.filepath.format(epoch=epoch + 1)
        save_weights(self.model, path)
        self.saved.append(path)

    def on_epoch_begin(self, epoch, logs=None):
        # keras sets the epoch used for '{epoch:02d}' at on_epoch_begin, so a fresh callback in a
        # fit(initial_epoch > 0) names its batch-count saves after the current epoch
        self._epoch = epoch

    def on_train_batch_end(self, batch, logs=None):
        self._batches += 1
        if self.save_freq != 'epoch' and self._batches % int(self.save_freq) == 0:
            self._save(self._epoch)

    def on_epoch_end(self, epoch, logs=None):
        if self.save_freq == 'epoch':
            self._save(epoch)


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch, self.history = [], {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


def _batches(data):
    return data() if callable(data) else data


def _rank(process_group):
    if process_group is None:
        return 0
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    grp = None if process_group is True else process_group
    return dist.get_rank(grp)


def _agree_stop(model, process_group):
    """Rank 0's stop_training decision on every rank (one broadcast of one int): a rank that
    stopped alone would leave the others blocked in the next train_step all-reduce."""
    if process_group is None:
        return
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    grp = None if process_group is True else process_group
    dev = getattr(model, 'device', None)
    if dist.get_backend(grp) == 'gloo' or dev is None:
        dev = torch.device('cpu')
    flag = torch.tensor([1 if getattr(model, 'stop_training', False) else 0], dtype=torch.int32, device=dev)
    src = dist.get_global_rank(grp, 0) if grp is not None else 0
    dist.broadcast(flag, src=src, group=grp)
    model.stop_training = bool(int(flag.item()))


def _agreed_batches(model, data, process_group, what):
    """The epoch's batches; data-parallel, every rank must run the same number of them (each
    train_step / test_step is a collective: a rank with more batches would block forever in its
    extra all-reduce). A source with len() is checked once per epoch (one all-reduce of two ints);
    any other source (a generator making a device tensor per batch) is streamed one batch at a time
    with a 'have another batch' flag all-reduced before each step, so the epoch is never held in
    memory at once. Either way a mismatch raises on every rank instead of hanging. Cost of the
    streamed form on NCCL: reading the flag back (int(n[0])) waits for the device, so each step's
    host enqueue starts only after the previous step finished — pass a source with len() (a list,
    a sized dataset) where that per-step sync matters."""
    batches = _batches(data)
    if process_group is None:
        return batches
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return batches
    grp = None if process_group is True else process_group
    dev = getattr(model, 'device', None)
    if dist.get_backend(grp) == 'gloo' or dev is None:
        dev = torch.device('cpu')

    def agree(k):
        n = torch.tensor([k, -k], dtype=torch.int64, device=dev)
        dist.all_reduce(n, op=dist.ReduceOp.MAX, group=grp)
        return int(n[0]), -int(n[1])

    def mismatch(lo, hi):
        return ValueError(f'data-parallel fit: ranks hold {lo}..{hi} {what} batches this epoch; every shard '
                          f'must have the same number of batches')

    if hasattr(batches, '__len__'):
        hi, lo = agree(len(batches))
        if hi != lo:
            raise mismatch(lo, hi)
        return batches

    def stream():
        it = iter(batches)
        done = object()
        count = 0
        while True:
            xy = next(it, done)
            hi, lo = agree(0 if xy is done else 1)
            if hi != lo:
                raise mismatch(count, count + 1)
            if xy is done:
                return
            count += 1
            yield xy
    return stream()


def fit(model, x, epochs=1, initial_epoch=0, validation_data=None, callbacks: Optional[List[Callback]] = None,
        verbose=0, process_group=None):
    """keras Model.fit over train_step / test_step. Logs per epoch: loss, z_loss, y_loss, detJ_loss
    (+ val_ prefixed on validation_data), host floats; per batch (on_train_batch_end) the same keys
    as 0-d device tensors (Callback). Returns a History.

    Data-parallel (process_group given, True = the default group): every rank passes its own
    shard of the batches; train_step and test_step all-reduce over the global batch, so the
    logged losses (and EarlyStopping's val_loss) are the same on every rank; rank 0's
    stop_training decision is broadcast after each epoch, and callbacks that write files
    (CSVLogger, ModelCheckpoint) run on rank 0 only. Every rank's shard must yield the same number
    of training (and validation) batches per epoch; a mismatch raises ValueError on every rank."""
    hist = History()
    rank = _rank(process_group)
    cbs = [cb for cb in list(callbacks or []) if rank == 0 or not cb.writes_files] + [hist]
    for cb in cbs:
        cb.set_model(model)
        cb.on_train_begin()
    model.stop_training = False
    for epoch in range(initial_epoch, epochs):
        for cb in cbs:
            cb.on_epoch_begin(epoch)
        for t in model.metrics:
            t.reset_state()
        logs = {}
        for i, xy in enumerate(_agreed_batches(model, x, process_group, 'training')):
            logs = model.train_step(xy, process_group=process_group)
            for cb in cbs:
                cb.on_train_batch_end(i, logs)
        logs = {k: float(v) for k, v in logs.items()}   # the epoch's one host read of the trackers
        if validation_data is not None:
            for t in model.metrics:
                t.reset_state()
            vlogs = {}
            for xy in _agreed_batches(model, validation_data, process_group, 'validation'):
                vlogs = model.test_step(xy, process_group=process_group)
            logs.update({'val_' + k: float(v) for k, v in vlogs.items()})
        if verbose and rank == 0:
            print(f'Epoch {epoch + 1}/{epochs} ' + ' - '.join(f'{k}: {v:.4f}' for k, v in logs.items()))
        for cb in cbs:
            cb.on_epoch_end(epoch, logs)
        _agree_stop(model, process_group)
        if model.stop_training:
            break
    return hist


def anneal_and_fit(model, xy_train: Iterable, xy_val: Optional[Iterable], num_annealing_epochs: int, num_epochs: int,
                   callbacks: Optional[List[Callback]] = None, seed: int = 0, verbose=0, process_group=None):
    """conv_cINN.py:583-636: anneal instance noise from pure noise (alpha = 0) towards clean data
    over num_annealing_epochs one-epoch fits, then fit the clean data up to num_epochs. Noise is
    redrawn every epoch (counter offsets advance per batch). As in the reference, each fit()
    starts with stop_training reset (keras), so an EarlyStopping that fires during annealing
    ends that one-epoch fit only and the schedule carries on. process_group: see fit (each rank
    passes its own shard; the noise is seeded per rank so shards draw independent noise)."""
    completed = 0
    hist = None
    rank = _rank(process_group)
    for i in range(int(num_annealing_epochs)):
        alpha = i / num_annealing_epochs
        if verbose and rank == 0:
            print(f'Annealing instance noise, alpha={alpha}, annealing epoch {i} of {num_annealing_epochs}.')

        def noisy(data, tag):
            def gen():
                off = 0
                for xy in _batches(data):
                    yield instance_noise(xy, alpha, seed=seed * 1000003 + 7919 * i + tag + 104729 * rank, offset=off)
                    off += xy.numel()
            return gen
        hist = fit(model, noisy(xy_train, 0), epochs=completed + 1, initial_epoch=completed,
                   validation_data=noisy(xy_val, 1) if xy_val is not None else None, callbacks=callbacks,
                   verbose=verbose, process_group=process_group)
        completed += 1
    return fit(model, xy_train, epochs=num_epochs, initial_epoch=completed, validation_data=xy_val,
               callbacks=callbacks, verbose=verbose, process_group=process_group)


def pretrain_on_noise(model, batch_size: int, num_epochs: int, batches_per_epoch: int = 20,
                      callbacks: Optional[List[Callback]] = None, seed: int = 0, verbose=0, process_group=None):
    """conv_pre_training_cINN_on_noise.py:100-147: condition the model on pure N(0, 1) inputs of its
    io_shape, `batches_per_epoch` batches per epoch (the reference's 20 * batch_size examples),
    fresh noise on every call (renew_noise); returns the History. process_group: data-parallel as
    in fit, batch_size images per rank, the noise seeded per rank."""
    import torch
    shape = (batch_size,) + tuple(model.io_shape)
    n_el = int(np.prod(shape))
    proto = torch.empty(shape, device=model.device, dtype=torch.float32)
    state = {'calls': 0}
    seed = seed + 104729 * _rank(process_group)

    def epoch_batches():
        c = state['calls']
        state['calls'] += 1
        for j in range(batches_per_epoch):
            yield renew_noise_like(proto, seed, (c * batches_per_epoch + j) * n_el)
    return fit(model, epoch_batches, epochs=num_epochs, callbacks=callbacks, verbose=verbose,
               process_group=process_group)


def renew_noise_like(t, seed, offset):
    from .base_functions import renew_noise
    return renew_noise(t, seed=seed, offset=offset)
