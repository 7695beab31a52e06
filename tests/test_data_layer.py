"""Dataset cache (``determined_1_amd/_data_layer.py``; reference ``harness/determined/_data_layer``)."""
import numpy as np
import torch

from determined_1_amd import _data_layer
from determined_1_amd.experimental import _local


class Squares(torch.utils.data.Dataset):
    calls = 0

    def __len__(self):
        return 10

    def __getitem__(self, i):
        Squares.calls += 1
        return {"x": torch.full((3,), float(i)), "y": torch.tensor(i * i)}


def make_env(tmp_path, total_batches=0, seed=7):
    cfg = {"hyperparameters": {"global_batch_size": 2}, "data_layer": {"type": "shared_fs",
           "container_storage_path": str(tmp_path)}, "reproducibility": {"experiment_seed": seed}}
    env, _, _ = _local.make_local_env(cfg)
    env.trial_seed = seed
    env.initial_workload.total_batches_processed = total_batches
    return env


def test_cache_written_once_and_reused(tmp_path):
    Squares.calls = 0
    env = make_env(tmp_path)
    ctx = _data_layer.DataLayerContext(env)
    stream = ctx.cache_validation_dataset("sq", "v1")(Squares)()
    assert Squares.calls == 10 and len(stream) == 10
    got = list(stream)
    assert [int(s["y"]) for s in got] == [i * i for i in range(10)]
    assert torch.equal(got[4]["x"], torch.full((3,), 4.0))
    ctx2 = _data_layer.DataLayerContext(env)
    list(ctx2.cache_validation_dataset("sq", "v1")(Squares)())
    assert Squares.calls == 10  # second trial memory-maps the cache
    assert (tmp_path / "sq" / "v1_val" / "meta.json").exists()


def test_train_stream_shards_shuffles_and_resumes(tmp_path):
    env = make_env(tmp_path)
    shards = []
    for rank in range(3):
        ctx = _data_layer.DataLayerContext(env, rank=rank, size=3)
        s = ctx.cache_train_dataset("sq", "v1", shuffle=True)(Squares)()
        assert len(s) == 3  # 10 // 3 with the remainder dropped
        it = iter(s)
        shards.append([int(next(it)["y"]) for _ in range(6)])  # repeats past one epoch
    first_epochs = sorted(v for sh in shards for v in sh[:3])
    assert first_epochs == sorted(i * i for i in range(9))
    # Resuming after 2 batches of 2 samples starts 4 samples into rank 0's stream.
    env2 = make_env(tmp_path, total_batches=2)
    s = _data_layer.DataLayerContext(env2, rank=0, size=3).cache_train_dataset("sq", "v1", shuffle=True)(Squares)()
    it = iter(s)
    assert [int(next(it)["y"]) for _ in range(2)] == shards[0][4:6]


def test_skip_shuffle_at_epoch_end_reuses_permutation(tmp_path):
    s = _data_layer.CachedStream(list(range(8)), shuffle=True, skip_shuffle_at_epoch_end=True, shuffle_seed=3)
    assert np.array_equal(s.epoch_keys(0), s.epoch_keys(5))
    s2 = _data_layer.CachedStream(list(range(8)), shuffle=True, shuffle_seed=3)
    assert not np.array_equal(s2.epoch_keys(0), s2.epoch_keys(1))


def test_trial_context_exposes_experimental(tmp_path):
    from determined_1_amd.pytorch import PyTorchTrialContext

    cfg = {"hyperparameters": {"global_batch_size": 4}, "data_layer": {"container_storage_path": str(tmp_path)}}
    ctx = PyTorchTrialContext.from_config(cfg)
    s = ctx.experimental.cache_train_dataset("sq", "v2")(Squares)()
    assert len(s) == 10 and ctx.experimental.get_train_cacheable().get_dataset_length() == 10


def _make_id_trial(storage):
    """PyTorchTrial over a cached dataset that records which sample ids it trains on."""
    from determined_1_amd import pytorch

    class Ids(torch.utils.data.Dataset):
        def __len__(self):
            return 24

        def __getitem__(self, i):
            return {"id": torch.tensor(i), "x": torch.full((2,), float(i))}

    class CachedIdTrial(pytorch.PyTorchTrial):
        seen = []

        def __init__(self, context):
            self.context = context
            self.model = context.wrap_model(torch.nn.Linear(2, 1))
            self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=0.01))

        def train_batch(self, batch, epoch_idx, batch_idx):
            CachedIdTrial.seen.append([int(v) for v in batch["id"]])
            loss = self.model(batch["x"]).pow(2).mean()
            self.context.backward(loss)
            self.context.step_optimizer(self.opt)
            return {"loss": loss}

        def evaluate_batch(self, batch):
            return {"validation_loss": self.model(batch["x"]).pow(2).mean()}

        def build_training_data_loader(self):
            @self.context.experimental.cache_train_dataset("ids", "v1", shuffle=True)
            def make():
                return Ids()

            return pytorch.DataLoader(make(), batch_size=self.context.get_per_slot_batch_size())

        def build_validation_data_loader(self):
            @self.context.experimental.cache_validation_dataset("ids", "v1")
            def make():
                return Ids()

            return pytorch.DataLoader(make(), batch_size=self.context.get_per_slot_batch_size())

    return CachedIdTrial


def test_pytorch_trial_trains_on_cached_dataset_and_resumes(tmp_path):
    """the data layer through a real PyTorchTrial -- cached map-style dataset, controller
    samplers shard/skip it, checkpoint + resume continues exactly where the first run stopped."""
    from tests.utils import Recorder, run

    trial = _make_id_trial(tmp_path)
    hp = {"global_batch_size": 4}
    extra = {"data_layer": {"type": "shared_fs", "container_storage_path": str(tmp_path / "cache")}}
    trial.seen = []
    run(trial, hp, Recorder().train(1, 3, 0).train(2, 3, 3), trial_seed=5, **extra)
    straight = list(trial.seen)
    assert len(straight) == 6
    first_epoch = sorted(i for b in straight for i in b)
    assert first_epoch == list(range(24))  # one pass over the (fixed-permuted) cache, no repeats
    assert [i for b in straight for i in b] != list(range(24))  # shuffle=True permuted it
    trial.seen = []
    ckpt = tmp_path / "ckpt"
    run(trial, hp, Recorder().train(1, 3, 0).checkpoint(1, 3, ckpt), trial_seed=5, **extra)
    trial.seen = []
    run(trial, hp, Recorder().train(2, 3, 3), load_path=ckpt, total_batches=3, trial_seed=5, **extra)
    assert trial.seen == straight[3:]
    assert not list((tmp_path / "cache" / "ids").glob(".tmp_*"))


def test_stale_writer_temp_dirs_removed(tmp_path):
    env = make_env(tmp_path)
    (tmp_path / "sq").mkdir()
    (tmp_path / "sq" / ".tmp_dead").mkdir()
    ctx = _data_layer.DataLayerContext(env, map_style=True)
    ds = ctx.cache_train_dataset("sq", "v9")(Squares)()
    assert isinstance(ds, _data_layer.CachedDataset) and len(ds) == 10
    assert not (tmp_path / "sq" / ".tmp_dead").exists()


def test_s3_data_layer_shares_cache_across_nodes(tmp_path):
    """data_layer type s3 (reference yogadl S3 storage): node A builds + uploads the cache (meta.json
    last), node B with its own local_cache_path downloads it and never runs the dataset builder."""
    from determined_1_amd.pytorch import PyTorchTrialContext
    from tests.test_storage_rest import AK, SK, S3Handler, _Server

    srv = _Server(S3Handler)
    srv.parts, srv.multipart_completed = {}, 0
    calls = []

    def make():
        calls.append(1)
        return Squares()

    try:
        for node in ("a", "b"):
            cfg = {"hyperparameters": {"global_batch_size": 4},
                   "data_layer": {"type": "s3", "bucket": "dl", "bucket_directory_path": "cache",
                                  "local_cache_path": str(tmp_path / node), "access_key": AK, "secret_key": SK,
                                  "endpoint_url": srv.url}}
            ctx = PyTorchTrialContext.from_config(cfg)
            s = ctx.experimental.cache_train_dataset("sq", "v3")(make)()
            assert len(s) == 10 and int(s[3]["y"]) == 9 and float(s[3]["x"][0]) == 3.0
        assert calls == [1]  # built once, on node a
        keys = sorted(srv.objects)
        assert "cache/sq/v3_train/meta.json" in keys and any(k.endswith(".npy") for k in keys)
        assert (tmp_path / "b" / "sq" / "v3_train" / "meta.json").exists()
    finally:
        srv.close()


def test_s3_data_layer_concurrent_same_node_readers(tmp_path):
    """Several ranks of one node miss the local cache at once: the download happens once,
    under the exclusive lock; no rank fails on the rename."""
    import threading

    from determined_1_amd.pytorch import PyTorchTrialContext
    from tests.test_storage_rest import AK, SK, S3Handler, _Server

    srv = _Server(S3Handler)
    srv.parts, srv.multipart_completed = {}, 0
    try:
        cfg = {"hyperparameters": {"global_batch_size": 4},
               "data_layer": {"type": "s3", "bucket": "dl", "bucket_directory_path": "cache",
                              "local_cache_path": str(tmp_path / "seed"), "access_key": AK, "secret_key": SK,
                              "endpoint_url": srv.url}}
        PyTorchTrialContext.from_config(cfg).experimental.cache_train_dataset("sq", "v4")(Squares)()
        cfg["data_layer"]["local_cache_path"] = str(tmp_path / "node")
        errors, sizes = [], []

        def rank():
            try:
                ctx = PyTorchTrialContext.from_config(cfg)
                sizes.append(len(ctx.experimental.cache_train_dataset("sq", "v4")(Squares)()))
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ts = [threading.Thread(target=rank) for _ in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not errors, errors
        assert sizes == [10] * 6
        assert not [p for p in (tmp_path / "node" / "sq").iterdir() if p.name.startswith(".tmp_")]
    finally:
        srv.close()
