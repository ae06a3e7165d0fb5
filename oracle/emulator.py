"""ORACLE (test infrastructure only): numpy restatement of the Zhao-Carr
microphysics emulator's inference graph (BASELINE config #5).

Reference (paths under /root/reference):
* model config                  projects/microphysics/train/dense.yaml:12-94
* transform_model               external/fv3fit/fv3fit/emulation/models/transformed_model.py:9-37
  (forward transforms, model, backward transforms on inputs + outputs)
* LogTransform                  external/fv3fit/fv3fit/emulation/transforms/transforms.py:111-129
  y = log(max(x, eps)); Difference backward: after = before + to  (transforms.py:18-58)
* MicrophysicsConfig.build      external/fv3fit/fv3fit/emulation/models/microphysics.py:100-136
  FieldInput: NormLayer.forward (x - center) / scale       (layers/fields.py:6-41,
                                                             layers/normalization2.py:20-24)
  combine_inputs: inputs sorted by name, concatenated      (layers/architecture.py:27-50)
  MLPBlock: depth x Dense(width, relu)                      (layers/architecture.py:228-272)
  StandardOutput: one linear Dense per output               (layers/architecture.py:296-333)
  FieldOutput: NormLayer.backward  y * scale + center      (layers/fields.py:44-66)
* normalisation fits: center per_feature mean, scale "all" = sqrt(mean over samples and
  features of (x - per-feature mean)^2)                     (normalization2.py:68-86)

``bf16=True`` rounds what the device kernel rounds (normalised inputs, hidden
activations and every weight to bfloat16, round-to-nearest-even; accumulation,
biases and the de-normalisation in float32) so the kernel can be checked at a
tight tolerance, and the plain float32/float64 graph gives the 1e-3 contract.
"""
import numpy as np


def to_bf16(x):
    """float32 -> nearest-even bfloat16, returned as float32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    b = x.view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(x), x, out)


def fit_center_per_feature(x):
    return x.astype(np.float64).mean(axis=0).astype(np.float32)


def fit_scale_all(x):
    mean = x.astype(np.float64).mean(axis=0)
    return np.float32(np.sqrt(((x.astype(np.float64) - mean) ** 2).mean()))


def model_inputs(raw, spec):
    """raw: name -> [ncol, nz] arrays; spec['features'] in model (sorted-name) order:
    dicts {name, source, log_eps or None}.  Returns the list of [ncol, nz] inputs."""
    out = []
    for f in spec["features"]:
        x = raw[f["source"]]
        if f.get("log_eps") is not None:
            x = np.log(np.maximum(x, np.asarray(f["log_eps"], x.dtype)))
        out.append(x)
    return out


def forward(raw, spec, params, dtype=np.float32, bf16=False):
    """-> dict of outputs: direct outputs and, for residual ones, the after-state."""
    rnd = to_bf16 if bf16 else (lambda a: a)
    xs = model_inputs({k: np.asarray(v, dtype) for k, v in raw.items()}, spec)
    feats = []
    for f, x in zip(spec["features"], xs):
        c = np.asarray(params["in_center"][f["name"]], dtype)
        s = np.asarray(params["in_scale"][f["name"]], dtype)
        feats.append((x - c) / s)
    h = rnd(np.concatenate(feats, axis=-1).astype(dtype))
    for W, b in zip(params["hidden_kernels"], params["hidden_biases"]):
        h = h @ rnd(np.asarray(W, dtype)) + np.asarray(b, dtype)
        h = rnd(np.maximum(h, 0))
    out = {}
    for o in spec["outputs"]:
        W = rnd(np.asarray(params["out_kernels"][o["name"]], dtype))
        y = h @ W + np.asarray(params["out_biases"][o["name"]], dtype)
        y = y * np.asarray(params["out_scale"][o["name"]], dtype) + np.asarray(params["out_center"][o["name"]], dtype)
        out[o["name"]] = y
        if o.get("residual_of"):
            out[o["after"]] = np.asarray(raw[o["residual_of"]], dtype) + y
    return out


# BASELINE config #5: projects/microphysics/train/dense.yaml
ZC_RAW = ["air_temperature_input", "specific_humidity_input", "cloud_water_mixing_ratio_input",
          "pressure_thickness_of_atmospheric_layer", "air_temperature_after_last_gscond",
          "specific_humidity_after_last_gscond"]


def zhao_carr_spec(nz=79):
    feats = [
        {"name": "air_temperature_input", "source": "air_temperature_input"},
        {"name": "specific_humidity_input", "source": "specific_humidity_input"},
        {"name": "cloud_water_mixing_ratio_input", "source": "cloud_water_mixing_ratio_input"},
        {"name": "log_cloud_input", "source": "cloud_water_mixing_ratio_input", "log_eps": 1e-10},
        {"name": "log_humidity_input", "source": "specific_humidity_input", "log_eps": 1e-8},
        {"name": "pressure_thickness_of_atmospheric_layer", "source": "pressure_thickness_of_atmospheric_layer"},
        {"name": "air_temperature_after_last_gscond", "source": "air_temperature_after_last_gscond"},
        {"name": "specific_humidity_after_last_gscond", "source": "specific_humidity_after_last_gscond"},
        {"name": "log_humidity_after_last_gscond", "source": "specific_humidity_after_last_gscond",
         "log_eps": 1e-8},
    ]
    feats = sorted(feats, key=lambda f: f["name"])  # combine_inputs: sorted by key
    outs = [
        {"name": "total_precipitation", "nz": 1},
        {"name": "cloud_precpd_difference", "nz": nz, "residual_of": "cloud_water_mixing_ratio_input",
         "after": "cloud_water_mixing_ratio_after_precpd"},
        {"name": "temperature_precpd_difference", "nz": nz, "residual_of": "air_temperature_input",
         "after": "air_temperature_after_precpd"},
        {"name": "humidity_precpd_difference", "nz": nz, "residual_of": "specific_humidity_input",
         "after": "specific_humidity_after_precpd"},
        {"name": "temperature_gscond_difference", "nz": nz, "residual_of": "air_temperature_input",
         "after": "air_temperature_after_gscond"},
        {"name": "humidity_gscond_difference", "nz": nz, "residual_of": "specific_humidity_input",
         "after": "specific_humidity_after_gscond"},
    ]
    return {"features": feats, "outputs": outs, "nz": nz, "width": 256, "depth": 2}


def synthetic_raw(ncol, nz=79, seed=0):
    """Physically plausible random column state (inputs of the emulator)."""
    rng = np.random.default_rng(seed)
    prof = np.linspace(200.0, 300.0, nz)[None, :]
    T = (prof + rng.normal(0, 5, (ncol, nz))).astype(np.float32)
    q = (0.02 * np.exp(-np.linspace(0, 6, nz))[None, :] * rng.uniform(0.2, 1.0, (ncol, nz))).astype(np.float32)
    qc = np.where(rng.uniform(size=(ncol, nz)) < 0.3, rng.uniform(0, 1e-4, (ncol, nz)), 0.0).astype(np.float32)
    delp = (np.linspace(200, 1800, nz)[None, :] * rng.uniform(0.98, 1.02, (ncol, nz))).astype(np.float32)
    return {
        "air_temperature_input": T,
        "specific_humidity_input": q,
        "cloud_water_mixing_ratio_input": qc,
        "pressure_thickness_of_atmospheric_layer": delp,
        "air_temperature_after_last_gscond": (T + rng.normal(0, 0.1, T.shape)).astype(np.float32),
        "specific_humidity_after_last_gscond": (q * rng.uniform(0.95, 1.05, q.shape)).astype(np.float32),
    }
