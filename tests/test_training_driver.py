"""Training driver (conv_cINN.py:517-641): fit / callbacks / annealed instance noise over the HIP
train_step. Callback logic is tested on CPU with a stub model; the end-to-end loop on the GPU."""
import math
import os

import numpy as np
import pytest
import torch

from arl_conditional_normalizing_flows_amd import training as T


class _Tracker:
    def __init__(self, name):
        self.name, self.v = name, 0.0

    def reset_state(self):
        self.v = 0.0

    def result(self):
        return self.v


class _Stub:
    """train_step returns a scripted val/train loss sequence (no GPU)."""

    def __init__(self, val_losses):
        self.metrics = [_Tracker('loss')]
        self.val = list(val_losses)
        self.epoch = -1
        self.steps = 0

    def train_step(self, xy, process_group=None):
        self.steps += 1
        return {'loss': 1.0}

    def test_step(self, xy):
        return {'loss': self.val[self.epoch]}

    def get_weights(self):
        return {'w': np.arange(3.0)}


class _EpochCounter(T.Callback):
    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_train_begin(self, logs=None):
        pass


def test_early_stopping_keras_semantics():
    stub = _Stub([5.0, 4.0, 4.5, 4.2, 3.0])
    es = T.EarlyStopping(monitor='val_loss', patience=2)

    class Bump(T.Callback):
        def on_train_batch_end(self, batch, logs=None):
            pass

    def data():
        stub.epoch += 1
        return [0]
    hist = T.fit(stub, data, epochs=5, validation_data=[0], callbacks=[es])
    # best 4.0 at epoch 1; epochs 2, 3 do not improve -> stop after epoch 3 (wait reaches 2)
    assert es.stopped_epoch == 3 and hist.epoch == [0, 1, 2, 3]
    assert hist.history['val_loss'] == [5.0, 4.0, 4.5, 4.2]


def test_csv_logger_sorted_header_and_append(tmp_path):
    p = str(tmp_path / 'hist.csv')
    stub = _Stub([2.0, 1.0, 0.5])

    def data():
        stub.epoch += 1
        return [0, 0]
    T.fit(stub, data, epochs=2, validation_data=[0], callbacks=[T.CSVLogger(p, append=True)])
    T.fit(stub, data, epochs=3, initial_epoch=2, validation_data=[0], callbacks=[T.CSVLogger(p, append=True)])
    rows = [r.strip().split(',') for r in open(p)]
    assert rows[0] == ['epoch', 'loss', 'val_loss'] and len(rows) == 4
    assert [r[0] for r in rows[1:]] == ['0', '1', '2'] and float(rows[3][2]) == 0.5


def test_model_checkpoint_batch_frequency(tmp_path):
    stub = _Stub([1.0] * 3)

    def data():
        stub.epoch += 1
        return [0, 0, 0]
    ck = T.ModelCheckpoint(str(tmp_path / 'ck.e{epoch:02d}.npz'), save_weights_only=True, save_freq=3)
    T.fit(stub, data, epochs=3, callbacks=[ck])
    assert [os.path.basename(p) for p in ck.saved] == ['ck.e01.npz', 'ck.e02.npz', 'ck.e03.npz']
    with np.load(ck.saved[0], allow_pickle=False) as z:
        assert np.array_equal(z['w'], np.arange(3.0))


@pytest.mark.gpu
def test_anneal_and_fit_end_to_end(gpu, tmp_path):
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    from arl_conditional_normalizing_flows_amd.optimizers import Adam
    from arl_conditional_normalizing_flows_amd.synthetic import class_batch
    cfg = PRESETS['small']
    flow = cFlow(**cfg.kwargs(), device=gpu)
    flow.set_weights(flow.initial_weights(3))
    flow.compile(optimizer=Adam(learning_rate=3e-4))
    H, W, D = cfg.io_shape
    train = [torch.from_numpy(class_batch(8, H, W, cfg.x_d, seed=s)).to(gpu) for s in range(3)]
    val = [torch.from_numpy(class_batch(8, H, W, cfg.x_d, seed=10))]
    val = [v.to(gpu) for v in val]
    csvp = str(tmp_path / 'h.csv')
    ck = T.ModelCheckpoint(str(tmp_path / 'w.e{epoch:02d}.npz'), save_freq=3)
    hist = T.anneal_and_fit(flow, train, val, num_annealing_epochs=2, num_epochs=5,
                            callbacks=[T.CSVLogger(csvp, append=True), ck, T.EarlyStopping(patience=10)])
    rows = list(open(csvp))
    assert len(rows) == 1 + 5                                    # 2 annealing + 3 clean epochs, one CSV
    assert all(math.isfinite(v) for v in hist.history['val_loss'])
    # clean-data training lowers the validation loss over its epochs
    assert hist.history['val_loss'][-1] < hist.history['val_loss'][0]
    # a checkpoint round-trips to identical parameters and outputs
    w_before = flow.params.detach().clone()
    T.load_weights(flow, ck.saved[-1])
    assert torch.equal(flow.params, w_before)


@pytest.mark.gpu
def test_pretrain_on_noise(gpu):
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    from arl_conditional_normalizing_flows_amd.optimizers import Adam
    cfg = PRESETS['tiny']
    flow = cFlow(**cfg.kwargs(), device=gpu)
    flow.set_weights(flow.initial_weights(1))
    flow.compile(optimizer=Adam(learning_rate=1e-3))
    hist = T.pretrain_on_noise(flow, batch_size=4, num_epochs=3, batches_per_epoch=4)
    losses = hist.history['loss']
    assert len(losses) == 3 and all(math.isfinite(v) for v in losses)
    assert losses[-1] < losses[0]
