"""Driver CLI surface (CPU): the reference's flags (train.py:49-55, train_lm.py:76-88, utils.py:60-70),
exp-dir naming (utils.py:310-367), model aliases and LM dispatch (train.py:107-134), loss curves
(utils.py:482-600)."""
import csv
import os
import textwrap

import pytest
import yaml

import train
import train_lm
import utils
from utils import FLAGS, get_exp_dir_path, load_config, maybe_make_dir, parse_flags, save_loss_curves

VIT_YAML = """\
seed: 0
print_progress: false
dataset: "tiny_imagenet_synthetic"
batch_size: 64
image_size: 64
num_epochs: 10
num_channels: 3
num_classes: 200
model: "vision_transformer"
vit_patch_size: 4
vit_hidden_size: 128
vit_mlp_dim: 256
vit_layers: 4
vit_heads: 4
vit_dropout: 0.1
vit_use_layernorm: true
vit_use_batchnorm: false
optim: muon
lr: 0.001
weight_decay: 0.01
beta1: 0.9
beta2: 0.9
muon_ns_coeffs: [3.4445, -4.7750, 2.0315]
eigen_tracking_enabled: true
hf_cg_tol: 1e-2
schedule_free: False
"""

LM_YAML = """\
seed: 0
matmul_precision: "highest"
seq_len: 2048
vocab_size: 50257
intra_doc_masking: True
model: "transformer"
d_model: 768
mlp_class: "glu"
expand: "8/3"
n_layers: 12
n_heads: 12
tie_embeddings: False
rope_theta: 500000.0
steps_budget: 12371
micro_batch_size: 16
grad_accumulation_steps: 8
dtype: "bfloat16"
optim: adam
lr: 3.e-4
weight_decay: 0.1
beta1: 0.9
beta2: 0.95
exp_name: "lm_fwedu_10BT"
out_dir: "./exp/llm"
"""


@pytest.fixture(autouse=True)
def _reset_flags():
    yield
    FLAGS.config = FLAGS.exp_name = FLAGS.job_idx = FLAGS.job_cluster = None


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(textwrap.dedent(text))
    return str(p)


@pytest.mark.parametrize("style", ["equals", "space"])
def test_flags_both_syntaxes(style):
    args = {"config": "c.yaml", "exp_name": "e1", "job_idx": "3", "job_cluster": "mi355x"}
    argv = [f"--{k}={v}" for k, v in args.items()] if style == "equals" else \
        [x for k, v in args.items() for x in (f"--{k}", v)]
    f = parse_flags(argv)
    assert (f.config, f.exp_name, f.job_idx, f.job_cluster) == ("c.yaml", "e1", 3, "mi355x")
    assert parse_flags([]).config == "config/config.yaml"


def test_vit_yaml_through_train_cli(tmp_path):
    path = _write(tmp_path, "config_vit.yaml", VIT_YAML)
    f = parse_flags([f"--config={path}"])
    cfg, n = load_config(f.config)
    assert n == 1 and cfg.lr == 1e-3 and cfg.hf_cg_tol == 1e-2 and cfg.schedule_free is False
    assert cfg.muon_ns_coeffs == [3.4445, -4.775, 2.0315]
    for alias in ("vit", "vit_small", "vision_transformer"):
        cfg.model = alias
        m = train.construct_model(cfg)
        assert (m.num_classes, m.hidden_size, m.num_layers) == (200, 128, 4)
    assert train.image_shape(cfg) == (64, 64, 64, 3)
    cfg.model = "resnet_small"
    with pytest.raises(ValueError, match="Unknown model"):
        train.construct_model(cfg)


def test_lm_yaml_through_both_clis(tmp_path, monkeypatch):
    path = _write(tmp_path, "lm_adam.yaml", LM_YAML)
    seen = []
    monkeypatch.setattr(train_lm, "run", lambda cfg: seen.append(("lm", cfg)) or "lm-state")
    # train.py hands model: transformer to train_lm.run (reference train.py:132-134)
    assert train.main([f"--config={path}"]) == "lm-state"
    assert train_lm.main(["--config", path, "--exp_name", "x"]) == "lm-state"
    assert [s[0] for s in seen] == ["lm", "lm"]
    cfg = seen[0][1]
    assert cfg.lr == 3e-4 and cfg.expand == "8/3" and cfg.micro_batch_size == 16 and cfg.intra_doc_masking is True
    assert FLAGS.exp_name == "x"


def test_exp_dir_rules(tmp_path):
    cfg = utils.Config(optim="muon", model="vit_small", out_dir=str(tmp_path))
    assert get_exp_dir_path(cfg) == os.path.join(str(tmp_path), "run_muon_vit_small")
    cfg.exp_name = "run"
    assert get_exp_dir_path(cfg).endswith("run_muon_vit_small")
    cfg.exp_name = "mine"
    assert get_exp_dir_path(cfg).endswith("mine")
    parse_flags(["--exp_name=flagged", "--job_idx=2"])
    d = get_exp_dir_path(cfg)
    assert d == os.path.join(str(tmp_path), "flagged", "job_idx_2")
    os.makedirs(d)
    open(os.path.join(d, "stale"), "w").close()
    maybe_make_dir(cfg)
    assert sorted(os.listdir(d)) == ["config.yaml"]
    assert yaml.safe_load(open(os.path.join(d, "config.yaml")))["exp_name"] == "mine"
    cfg.over_write = False
    with pytest.raises(ValueError, match="existing exp_dir"):
        maybe_make_dir(cfg)


def test_sweep_job_idx_from_flags(tmp_path):
    path = _write(tmp_path, "sweep.yaml", "lr: [1e-3, 3e-4]\nb: [1, 2, 3]\nmodel: vit\n")
    parse_flags([f"--config={path}", "--job_idx=4"])
    cfg, n = load_config(path)
    assert n == 6 and cfg.lr == 3e-4 and cfg.b == 2


def test_save_loss_curves(tmp_path):
    cfg = utils.Config(optim="soap", model="vit", out_dir=str(tmp_path), exp_name="c")
    save_loss_curves(cfg, "soap", [1.0, 2.5], [1, 2], [2.0, 1.5], [2.1, 1.7], [0.1, 0.3], [0.1, 0.2])
    d = get_exp_dir_path(cfg)
    rows = list(csv.reader(open(os.path.join(d, "soap_metrics.csv"))))
    assert rows[0] == ["iteration", "wall_time_sec", "train_loss", "eval_loss", "train_accuracy", "eval_accuracy"]
    assert rows[2] == ["2", "2.5", "1.5", "1.7", "0.3", "0.2"]
    for kind in ("time", "iter"):
        png = os.path.join(d, f"soap_{kind}_vs_eval_loss.png")
        assert open(png, "rb").read(8) == b"\x89PNG\r\n\x1a\n"
    with pytest.raises(ValueError, match="same length"):
        save_loss_curves(cfg, "soap", [1.0], [1, 2], [2.0, 1.5], [2.1, 1.7], [0.1, 0.3], [0.1, 0.2])


@pytest.mark.parametrize("keys,world,ok,use", [({}, 1, True, False), ({}, 4, True, True),
                                               ({"use_pmap": True}, 1, True, False),
                                               ({"use_pmap": True}, 2, True, True),
                                               ({"use_pmap": False}, 1, True, False),
                                               ({"use_pmap": False}, 2, False, None),
                                               ({"force_single_device": True}, 8, False, None),
                                               ({"force_single_device": True}, 1, True, False)])
def test_use_pmap_force_single_device(keys, world, ok, use):
    """train_lm.py:476-483: the keys decide DP; a single-device request under N > 1 ranks is refused."""
    from plaincv_amd.engine.data_parallel import resolve_use_dp
    from utils import Config
    cfg = Config(model="transformer", **keys)
    if ok:
        assert resolve_use_dp(cfg, world) is use
    else:
        with pytest.raises(ValueError, match="single-device"):
            resolve_use_dp(cfg, world)


def test_batchnorm_vit_config_runs_fp32():
    """vit_use_batchnorm configs build the fp32 runner (the reference BN ViT's precision) unless
    vit_dtype asks for bf16; an unknown vit_dtype is refused."""
    from utils import Config
    base = dict(model="vit_small", dataset="fashion_mnist", vit_use_layernorm=False, vit_use_batchnorm=True)
    assert train.construct_model(Config(**base)).dtype == "float32"
    assert train.construct_model(Config(vit_dtype="bfloat16", **base)).dtype == "bfloat16"
    with pytest.raises(ValueError, match="vit_dtype"):
        train.construct_model(Config(vit_dtype="float16", **base))
