"""BERT SQuAD trial (examples/nlp/bert_squad_pytorch, BASELINE config #5's trial) through the
PyTorchTrial controller: checkpoint + restore mid-training with aggregation_frequency 2 continues
exactly like an uninterrupted run (optimizer moments, the LambdaLR step, the partial aggregation
boundary, data position), on a tiny encoder so it runs on CPU.

Reference: harness/tests/experiment/utils.py:365 (checkpoint-restore equivalence) and
examples/nlp/bert_squad_pytorch/distributed.yaml (aggregation_frequency, AdamW, clipping)."""
import os
import pathlib

import numpy as np
import pytest

from determined_1_amd.experimental import load_model_def
from tests.utils import Recorder, run

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HP = {"global_batch_size": 4, "max_seq_length": 32, "hidden_size": 64, "num_hidden_layers": 2,
      "num_attention_heads": 4, "intermediate_size": 128, "vocab_size": 512, "amp": "O0", "learning_rate": 1e-3,
      "num_warmup_steps": 2, "num_training_steps": 40, "max_grad_norm": 1.0, "weight_decay": 0.01,
      "train_records": 64, "validation_records": 8}


def _trial():
    return load_model_def(os.path.join(REPO, "examples", "nlp", "bert_squad_pytorch")).BertSQuADTrial


def _losses(resp, i):
    return [float(m["loss"]) for m in resp[i]["metrics"]["batch_metrics"]]


@pytest.mark.parametrize("agg", [1, 2])
def test_bert_checkpoint_restore_equivalence(tmp_path: pathlib.Path, agg):
    trial = _trial()
    opt = {"aggregation_frequency": agg}
    # 6 batches straight
    _, ra = run(trial, HP, Recorder().train(1, 3, 0).train(2, 3, 3), trial_seed=5, optimizations=opt)
    # 3 batches, checkpoint (mid aggregation window when agg == 2), restore, 3 more
    ckpt = tmp_path / "ckpt"
    _, rb = run(trial, HP, Recorder().train(1, 3, 0).checkpoint(1, 3, ckpt), trial_seed=5, optimizations=opt)
    assert (ckpt / "state_dict.pth").exists()
    np.testing.assert_allclose(_losses(rb, 0), _losses(ra, 0), rtol=0, atol=0)
    _, rc = run(trial, HP, Recorder().train(2, 3, 3), load_path=ckpt, total_batches=3, trial_seed=5,
                optimizations=opt)
    a2, c2 = _losses(ra, 1), _losses(rc, 0)
    assert len(a2) == len(c2) == 3
    np.testing.assert_allclose(c2, a2, rtol=1e-6, atol=1e-7)
    # the run trains: loss moves
    assert a2[-1] != _losses(ra, 0)[0]


@pytest.mark.gpu
def test_bert_checkpoint_restore_equivalence_gpu_o2(tmp_path: pathlib.Path, gpu):
    """The same on the GPU at O2 (fp32 master weights in the fused arena optimizer, GradSink
    gradient landing, MFMA attention), checkpointed inside an aggregation window of 2."""
    trial = _trial()
    hp = dict(HP, amp="O2", max_seq_length=64)
    opt = {"aggregation_frequency": 2}
    _, ra = run(trial, hp, Recorder().train(1, 3, 0).train(2, 3, 3), trial_seed=5, optimizations=opt, use_gpu=True)
    ckpt = tmp_path / "ckpt"
    run(trial, hp, Recorder().train(1, 3, 0).checkpoint(1, 3, ckpt), trial_seed=5, optimizations=opt, use_gpu=True)
    _, rc = run(trial, hp, Recorder().train(2, 3, 3), load_path=ckpt, total_batches=3, trial_seed=5,
                optimizations=opt, use_gpu=True)
    np.testing.assert_allclose(_losses(rc, 0), _losses(ra, 1), rtol=1e-5, atol=1e-6)


def test_dropout_rng_stream_is_trial_state():
    """The native dropout (seed, offset) stream restarts when the trial seeds torch and round-trips
    through rng_state / set_rng_state (what the checkpoint stores)."""
    import torch

    from determined_1_amd.ops import transformer as tf
    from determined_1_amd.pytorch._trial import PyTorchTrialController

    PyTorchTrialController._set_random_seeds(11)
    a = [tf.next_rng() for _ in range(3)]
    st = tf.rng_state()
    b = [tf.next_rng() for _ in range(2)]
    tf.set_rng_state(st)
    assert [tf.next_rng() for _ in range(2)] == b
    PyTorchTrialController._set_random_seeds(11)
    assert [tf.next_rng() for _ in range(3)] == a and a[0][0] == torch.initial_seed()
    assert [o for _, o in a] == [1, 2, 3]


@pytest.mark.gpu
def test_hip_graph_replays_draw_fresh_dropout_masks(gpu):
    """The native dropout kernels take (seed, offset) as kernel arguments, which a hipGraph replay
    repeats; the captured step bumps a device offset counter the kernels add, so the BERT trial runs
    as graph replays (no eager fallback) and every replay draws new masks -- the counter equals the
    replay count, and a different counter value gives a different mask."""
    import torch

    from determined_1_amd.ops import transformer as tf

    trial = _trial()
    hp = dict(HP, amp="O2", max_seq_length=64)
    ctrl, _ = run(trial, hp, Recorder().train(1, 6, 0), trial_seed=5, optimizations={"hip_graph": True}, use_gpu=True)
    g = ctrl._graph
    assert g is not None and g.disabled_reason is None and g.replays >= 3, (g.disabled_reason, g.replays)
    idx = torch.cuda.current_device()
    assert int(tf._RNG_BASE[idx].item()) >= g.replays
    m0 = tf.dropout_mask(4096, 0.1, 123, 7, gpu)
    tf._RNG_BASE[idx].add_(1)
    m1 = tf.dropout_mask(4096, 0.1, 123, 7, gpu)
    tf._RNG_BASE[idx].sub_(1)
    assert not torch.equal(m0, m1)
