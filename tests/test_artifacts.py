"""Model artifacts: PytorchPredictor's scalers.zip and a weights-only
column MLP (external/fv3fit/fv3fit/pytorch/predict.py:40-57, 60-120, 274-387), and the
Keras DenseModel exporter's writer (tools/export_keras_dense.py)."""
import io
import os
import sys
import zipfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _scalers(rng, nz=79):
    from fv3net_amd.normalization import StandardScaler

    out = {}
    for name, loc, scale, n in (("air_temperature", 260, 15, nz), ("specific_humidity", 0.01, 0.005, nz),
                                ("surface_pressure", 1e5, 1e3, None),
                                ("dQ1", 0, 1e-4, nz), ("dQ2", 0, 3e-8, nz), ("precip", 0, 1e-3, None)):
        s = StandardScaler()
        s.fit(rng.normal(loc, scale, (500, n) if n else (500,)))
        out[name] = s
    return out


def test_scalers_zip_round_trip():
    """dump_mapping/load_mapping: a zip with one npz per variable (predict.py:40-57)."""
    from fv3net_amd.pytorch_predictor import dump_mapping, load_mapping
    from fv3net_amd.normalization import StandardScaler

    sc = _scalers(np.random.default_rng(0))
    buf = io.BytesIO()
    dump_mapping(sc, buf)
    buf.seek(0)
    with zipfile.ZipFile(buf) as z:
        assert sorted(z.namelist()) == sorted(sc)
        arr = np.load(z.open("air_temperature"), allow_pickle=False)
        np.testing.assert_array_equal(arr["mean"], sc["air_temperature"].mean)
    buf.seek(0)
    loaded = load_mapping(StandardScaler, buf)
    assert loaded == sc


def _mlp(k_in, k_out, width=32, seed=0):
    import torch

    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(k_in, width), torch.nn.ReLU(), torch.nn.Linear(width, width),
                               torch.nn.ReLU(), torch.nn.Linear(width, k_out))


def _dump_pytorch_dir(path, model, scalers, ins, outs, whole_module=False):
    import torch
    import yaml

    from fv3net_amd.pytorch_predictor import dump_mapping

    os.makedirs(path, exist_ok=True)
    torch.save(model if whole_module else model.state_dict(), os.path.join(path, "weight.pt"))
    with open(os.path.join(path, "scalers.zip"), "wb") as f:
        dump_mapping(scalers, f)
    with open(os.path.join(path, "config.yaml"), "w") as f:
        yaml.safe_dump({"input_variables": ins, "output_variables": outs}, f)
    with open(os.path.join(path, "name"), "w") as f:
        f.write("pytorch_predictor")


def test_pickled_module_is_refused(tmp_path):
    """The reference pickles the nn.Module; only a weights-only state dict is read."""
    from fv3net_amd.predictor import load

    sc = _scalers(np.random.default_rng(1))
    ins, outs = ["air_temperature", "specific_humidity", "surface_pressure"], ["dQ1", "dQ2", "precip"]
    _dump_pytorch_dir(str(tmp_path), _mlp(159, 159), sc, ins, outs, whole_module=True)
    with pytest.raises(ValueError, match="weights-only"):
        load(str(tmp_path))


def test_keras_exporter_writer_round_trip(tmp_path):
    """write_predictor on Keras-layout arrays -> the mi355x-dense directory -> load."""
    from export_keras_dense import write_predictor
    from fv3net_amd.predictor import DenseColumnPredictor, load

    rng = np.random.default_rng(2)
    k_in = 79 + 70  # q clipped to levels 9..79
    params = {"hidden_kernels": [rng.normal(size=(k_in, 64)), rng.normal(size=(64, 64))],
              "hidden_biases": [rng.normal(size=64), rng.normal(size=64)],
              "out_kernels": [rng.normal(size=(64, 79)), rng.normal(size=(64, 79))],
              "out_biases": [rng.normal(size=79), rng.normal(size=79)],
              "in_mean": [rng.normal(size=79), rng.normal(size=70)],
              "in_sigma": [rng.uniform(1, 2, 79), rng.uniform(1, 2, 70)],
              "out_mean": [rng.normal(size=79), rng.normal(size=79)],
              "out_sigma": [rng.uniform(1, 2, 79), rng.uniform(1, 2, 79)]}
    write_predictor(str(tmp_path), ["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [79, 79], [79, 79],
                    params, 1e-7, clip={"specific_humidity": (9, None)}, output_limits={"dQ2": (None, 1e-3)})
    with open(tmp_path / "name") as f:
        assert f.read().strip() == "mi355x-dense"
    pred = load(str(tmp_path))
    assert isinstance(pred, DenseColumnPredictor)
    cfg, p = pred.model.config, pred.model.params
    assert cfg.width == 64 and cfg.depth == 3 and cfg.clip == {"specific_humidity": (9, None)}
    assert cfg.output_limits == {"dQ2": (None, 1e-3)}
    for k, v in params.items():
        for a, b in zip(p[k], v):
            np.testing.assert_array_equal(a, np.asarray(b, np.float32))


@pytest.mark.gpu
def test_pytorch_column_predictor_matches_torch(gpu, tmp_path):
    """Loaded through the name-file registry: pack (float64 normalisation -> float32), the
    MLP on the fused kernel, float64 unpack; against the same arithmetic with the MLP in
    float64 on the CPU, per output variable within 1e-5 of its scale."""
    import torch

    from fv3net_amd import dataset as D
    from fv3net_amd.predictor import load

    rng = np.random.default_rng(3)
    sc = _scalers(rng)
    ins, outs = ["air_temperature", "specific_humidity", "surface_pressure"], ["dQ1", "dQ2", "precip"]
    model = _mlp(79 + 79 + 1, 79 + 79 + 1)
    _dump_pytorch_dir(str(tmp_path), model, sc, ins, outs)
    pred = load(str(tmp_path))
    nt, nx, ny = 6, 12, 12
    X = {"air_temperature": rng.normal(260, 15, (nt, nx, ny, 79)),
         "specific_humidity": rng.normal(0.01, 0.005, (nt, nx, ny, 79)),
         "surface_pressure": rng.normal(1e5, 1e3, (nt, nx, ny))}
    ds = D.Dataset({"air_temperature": D.DataArray(torch.from_numpy(X["air_temperature"]).cuda(),
                                                   ("tile", "x", "y", "z")),
                    "specific_humidity": D.DataArray(torch.from_numpy(X["specific_humidity"]).cuda(),
                                                     ("tile", "x", "y", "z")),
                    "surface_pressure": D.DataArray(torch.from_numpy(X["surface_pressure"]).cuda(),
                                                    ("tile", "x", "y"))})
    out = pred.predict(ds)
    # the reference's pack -> model -> unpack, the model in float64 on the host
    cols = []
    for n in ins:
        x = X[n].reshape(nt * nx * ny, -1)
        cols.append(((x - sc[n].mean) / sc[n].std).astype(np.float32))
    packed = np.concatenate(cols, axis=1).astype(np.float64)
    with torch.no_grad():
        y = model.double()(torch.from_numpy(packed)).numpy()
    off = 0
    for n in outs:
        nf = 79 if np.ndim(sc[n].mean) else 1
        ref = y[:, off:off + nf] * sc[n].std + sc[n].mean
        off += nf
        got = out[n].data.cpu().numpy()
        assert out[n].dims == (("tile", "x", "y", "z") if nf > 1 else ("tile", "x", "y"))
        got = got.reshape(nt * nx * ny, nf)
        err = np.abs(got - ref) / (np.abs(ref - sc[n].mean).max(axis=0) + 1e-30)
        assert err.max() < 1e-5, (n, err.max())


def _training_config_from_spec(spec):
    """A microphysics TrainConfig (train_microphysics.py:127-166, the dense.yaml shape)
    rebuilt from the emulator restatement's spec (oracle/emulator.py): the model inputs
    in a scrambled order, a LogTransform entry per log feature, a Difference entry per
    after-state output."""
    tt = []
    for f in spec["features"]:
        if f.get("log_eps"):
            tt.append({"to": f["name"], "source": f["source"], "transform": {"epsilon": f["log_eps"]}})
    for o in spec["outputs"]:
        if o.get("after"):
            tt.append({"to": o["name"], "before": o["residual_of"], "after": o["after"]})
    names = [f["name"] for f in spec["features"]]
    return {"tensor_transform": tt,
            "model": {"architecture": {"name": "dense", "kwargs": {"width": 256, "depth": 2}},
                      "input_variables": names[::-1],
                      "direct_out_variables": [o["name"] for o in spec["outputs"]]}}


def test_emulator_training_config_parse():
    """fv3net_amd.emulator.features_outputs_from_config on a training configuration
    gives the product's Zhao-Carr features and outputs (sorted inputs, LogTransform
    sources and epsilons, Difference before / after), as the restatement specifies."""
    from fv3net_amd import emulator as E
    from oracle import emulator as OE

    spec = OE.zhao_carr_spec()
    feats, outs = E.features_outputs_from_config(_training_config_from_spec(spec), {"total_precipitation": 1})
    assert feats == E.zhao_carr_features()
    assert outs == E.zhao_carr_outputs()
    with pytest.raises(NotImplementedError):
        E.features_outputs_from_config({"tensor_transform": [{"to": "x", "before": "a", "after": "b"}],
                                        "model": {"input_variables": ["x"]}}, {})


def test_emulator_dict_exporter_writer_round_trip(tmp_path):
    """write_emulator_predictor (the all-keras-dict path of tools/export_keras_dense.py
    after the TF read) -> an mi355x-dense directory with input sources -> load: raw
    variables in, after-states out, the weights and scalar norm scales broadcast per
    level, the bf16x3 precision kept."""
    from export_keras_dense import write_emulator_predictor
    from fv3net_amd.emulator import MicrophysicsEmulator
    from fv3net_amd.predictor import DenseColumnPredictor, load
    from oracle import emulator as OE

    spec = OE.zhao_carr_spec(nz=12)
    cfg = _training_config_from_spec(spec)
    rng = np.random.default_rng(3)
    nz, w = 12, 32
    feats = [f["name"] for f in spec["features"]]
    outs = {o["name"]: o["nz"] for o in spec["outputs"]}
    params = {"hidden_kernels": [rng.normal(size=(nz * len(feats), w)), rng.normal(size=(w, w))],
              "hidden_biases": [rng.normal(size=w), rng.normal(size=w)],
              "in_center": {n: rng.normal(size=nz) for n in feats},
              "in_scale": {n: np.float32(rng.uniform(1, 2)) for n in feats},
              "out_kernels": {n: rng.normal(size=(w, k)) for n, k in outs.items()},
              "out_biases": {n: rng.normal(size=k) for n, k in outs.items()},
              "out_center": {n: rng.normal(size=k) for n, k in outs.items()},
              "out_scale": {n: np.float32(rng.uniform(1, 2)) for n, k in outs.items()}}
    write_emulator_predictor(str(tmp_path), cfg, outs, nz, params)
    pred = load(str(tmp_path))
    assert isinstance(pred, DenseColumnPredictor)
    # the raw variables, each once, in the order the sorted features first read them
    assert pred.input_variables == list(dict.fromkeys(f["source"] for f in spec["features"]))
    assert len(pred.input_variables) == 6
    assert pred.output_variables[0] == "total_precipitation"
    assert pred.output_variables[1:] == [o["after"] for o in spec["outputs"][1:]]
    assert pred.model.precision == "bf16x3"
    emu = MicrophysicsEmulator.from_predictor(pred)
    assert [(f.name, f.source, f.log_eps) for f in emu.features] == \
        [(f["name"], f["source"], f.get("log_eps")) for f in spec["features"]]
    p = emu.params_by_name()
    for n in feats:
        np.testing.assert_array_equal(p["in_center"][n], np.asarray(params["in_center"][n], np.float32))
        assert p["in_scale"][n] == params["in_scale"][n]
    for o in spec["outputs"]:
        key = o.get("after") or o["name"]
        np.testing.assert_array_equal(p["out_kernels"][key], np.asarray(params["out_kernels"][o["name"]], np.float32))
