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


@pytest.mark.parametrize("agg,amp", [(1, "O0"), (2, "O0"), (2, "O2")])
def test_bert_checkpoint_restore_equivalence(tmp_path: pathlib.Path, agg, amp):
    """O2 (bf16 parameters, fp32 moments and master weights in the fused arenas) resumes exactly too:
    torch's Optimizer.load_state_dict casts floating state to the parameter dtype, which rounded the
    moments and masters to bf16 on every restore (ops/optim.py keeps the saved precision)."""
    trial = _trial()
    HP_ = dict(HP, amp=amp)
    opt = {"aggregation_frequency": agg}
    # 6 batches straight
    _, ra = run(trial, HP_, Recorder().train(1, 3, 0).train(2, 3, 3), trial_seed=5, optimizations=opt)
    # 3 batches, checkpoint (mid aggregation window when agg == 2), restore, 3 more
    ckpt = tmp_path / "ckpt"
    _, rb = run(trial, HP_, Recorder().train(1, 3, 0).checkpoint(1, 3, ckpt), trial_seed=5, optimizations=opt)
    assert (ckpt / "state_dict.pth").exists()
    np.testing.assert_allclose(_losses(rb, 0), _losses(ra, 0), rtol=0, atol=0)
    _, rc = run(trial, HP_, Recorder().train(2, 3, 3), load_path=ckpt, total_batches=3, trial_seed=5,
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
def test_graph_replays_draw_fresh_native_dropout_masks(gpu):
    """The native dropout kernels take (seed, offset) as kernel arguments, which a hipGraph replay
    repeats; they add a device offset counter that a captured step bumps first (what the hipGraph
    trial builder does), so two replays draw different masks, each equal to the eager kernel at that
    counter value."""
    import torch

    from determined_1_amd.ops import transformer as tf

    g0 = torch.Generator(device="cpu").manual_seed(3)
    h = torch.randn(512, 64, generator=g0).to(gpu, torch.bfloat16)
    gamma = torch.ones(64, device=gpu, dtype=torch.bfloat16)
    beta = torch.zeros(64, device=gpu, dtype=torch.bfloat16)
    tf._ln_forward(h, None, gamma, beta, 0.5, 1e-5)  # eager first: the counter exists before capture
    idx = torch.cuda.current_device()
    base0 = int(tf._RNG_BASE[idx].item())
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            tf.bump_rng_base()
            y, _, _, seed, off = tf._ln_forward(h, None, gamma, beta, 0.5, 1e-5)
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    y1 = y.clone()
    graph.replay()
    y2 = y.clone()
    torch.cuda.synchronize()
    assert int(tf._RNG_BASE[idx].item()) == base0 + 2
    assert not torch.equal(y1, y2)
    # replay 2 == the eager kernel with the counter at base0 + 2 and the captured (seed, offset)
    state = tf.rng_state()
    tf.set_rng_state({"seed": seed, "offset": off, "base": {idx: base0 + 2}})
    y_eager, _, _, _, _ = tf._ln_forward(h, None, gamma, beta, 0.5, 1e-5)
    tf.set_rng_state(state)
    assert torch.equal(y_eager, y2)
