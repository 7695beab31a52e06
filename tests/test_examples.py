"""Every official example's configs validate and its trial passes local test mode on CPU
(reference ``examples/tests/test_official.py``).  Heavy models are shrunk through hparam
overrides so the test stays CPU-sized."""
import pathlib

import pytest
import yaml

from determined_1_amd.config import merge_with_defaults, validate_experiment_config
from determined_1_amd.experimental import run_local_test

EX = pathlib.Path(__file__).resolve().parent.parent / "examples"
CONFIGS = sorted(EX.rglob("*.yaml"))
SHRINK = {
    "resnet50_pytorch": {"arch": "resnet18", "image_size": 32, "num_classes": 10, "global_batch_size": 2,
                         "train_records": 16, "validation_records": 4, "amp": "O0", "channels_last": False},
    "bert_squad_pytorch": {"num_hidden_layers": 1, "hidden_size": 64, "num_attention_heads": 2,
                           "intermediate_size": 128, "max_seq_length": 128, "global_batch_size": 2,
                           "train_records": 8, "validation_records": 4, "amp": "O2"},
    "albert_squad_pytorch": {"num_hidden_layers": 2, "hidden_size": 64, "num_attention_heads": 2,
                             "intermediate_size": 128, "embedding_size": 16, "vocab_size": 2000,
                             "max_seq_length": 128, "global_batch_size": 2, "train_records": 8,
                             "validation_records": 4, "amp": "O2"},
    "bert_glue_pytorch": {"num_hidden_layers": 1, "hidden_size": 64, "num_attention_heads": 2,
                          "intermediate_size": 128, "vocab_size": 2000, "max_seq_length": 64, "global_batch_size": 2,
                          "train_records": 8, "validation_records": 4, "amp": "O2"},
    "protonet_omniglot_pytorch": {"num_classes_train": 5, "num_classes_val": 5, "hidden_dim": 16, "embedding_dim": 16,
                                  "tasks_per_epoch_train": 4, "tasks_per_epoch_val": 2, "num_glyph_classes": 40},
    "darts_cifar10_pytorch": {"init_channels": 8, "layers": 5, "global_batch_size": 2, "train_records": 8,
                              "validation_records": 4},
    "darts_penntreebank_pytorch": {"emsize": 32, "nhid": 32, "nhidlast": 32, "vocab_size": 200, "train_tokens": 4000,
                                   "valid_tokens": 800, "global_batch_size": 4, "eval_batch_size": 4, "bptt": 10,
                                   "max_seq_length_delta": 4},
    "search": {"init_channels": 8, "layers": 3, "nodes": 2, "global_batch_size": 2, "train_records": 8,
               "validation_records": 4},  # nas/gaea_pytorch/search
    "eval": {"num_classes": 10, "image_size": 32, "init_channels": 8, "layers": 3, "global_batch_size": 2,
             "train_records": 8, "validation_records": 4},  # nas/gaea_pytorch/eval
    "cifar10_pytorch": {"amp": "O0", "global_batch_size": 4, "validation_records": 64},  # not the 10k test split
    "mnist_pytorch": {"global_batch_size": 4, "validation_records": 64},  # not the 10k test split
    "fasterrcnn_coco_pytorch": {"backbone": "resnet26", "num_images": 10, "min_image_size": 60, "max_image_size": 90,
                                "transform_min_size": 96, "transform_max_size": 160},
    "detr_coco_pytorch": {"backbone": "resnet26", "enc_layers": 1, "dec_layers": 2, "hidden_dim": 32, "nheads": 2,
                          "dim_feedforward": 64, "num_queries": 10, "min_image_size": 64, "max_image_size": 96,
                          "train_records": 8, "validation_records": 4, "num_workers": 0, "global_batch_size": 2},
    "gan_mnist_pytorch": {"global_batch_size": 4},
    "retinanet_coco_pytorch": {"backbone": "resnet26", "train_records": 6, "validation_records": 2,
                               "min_image_size": 60, "max_image_size": 90, "transform_min_size": 96,
                               "transform_max_size": 160, "num_classes": 5, "global_batch_size": 2},
    "maskrcnn_coco_pytorch": {"backbone": "resnet26", "train_records": 6, "validation_records": 2,
                              "min_image_size": 60, "max_image_size": 90, "transform_min_size": 96,
                              "transform_max_size": 160, "num_classes": 5, "global_batch_size": 2,
                              "mask_bucket": 8},
}


@pytest.mark.parametrize("cfg_path", CONFIGS, ids=lambda p: f"{p.parent.name}/{p.name}")
def test_example_config_validates(cfg_path):
    cfg = yaml.safe_load(cfg_path.read_text())
    assert validate_experiment_config(merge_with_defaults(cfg)) == []


@pytest.mark.parametrize("example", sorted({p.parent for p in CONFIGS}), ids=lambda p: p.name)
def test_example_local_test_mode(example):
    const = example.joinpath("const.yaml")
    if not const.exists():
        const = example.joinpath("const_fake.yaml")  # reference name for the no-download config
    cfg = yaml.safe_load(const.read_text())
    hp = {}
    for k, v in cfg["hyperparameters"].items():
        hp[k] = v["val"] if isinstance(v, dict) and v.get("type") == "const" else v
    hp.update(SHRINK.get(example.name, {}))
    cfg["hyperparameters"] = hp
    run_local_test(cfg, str(example))
