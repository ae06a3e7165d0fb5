"""The reference's StandardNormLayer / StandardDenormLayer known-answer test
(external/fv3fit/tests/emulation/layers/test_normalization.py:27-53), run through the
oracle (CPU) and through the fused dense kernel (GPU).

Input [[0, 0], [1, 2]] (2 samples x 2 features); fitted mean [0.5, 1], population std
[0.5, 1]; normalised [[-1, -1], [1, 1]] (rtol 1e-6); denormalising that gives the input
back (rtol 1e-6, atol 1e-6).  To expose the kernel's normalised stage, the network is a
relu-pair identity: hidden W1 = [I, -I] (units x, -x, then zeros), output
W_out = [I; -I] so y = relu(x) - relu(-x) = x.  With output mean 0 / sigma 1 the kernel
returns the normalised values; with the fitted mean / sigma it returns norm -> denorm.
"""
import numpy as np
import pytest

from oracle.dense import dense_predict

X = np.array([[0.0, 0.0], [1.0, 2.0]], np.float32)
NORM = np.array([[-1.0, -1.0], [1.0, 1.0]])
WIDTH = 64


def _model(denorm: bool):
    from fv3net_amd import normalization
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    mean, std = normalization.fit_mean_std(X)
    k1 = np.zeros((2, WIDTH), np.float32)
    k1[0, 0] = k1[1, 1] = 1.0
    k1[0, 2] = k1[1, 3] = -1.0
    k2 = np.zeros((WIDTH, 2), np.float32)
    k2[0, 0] = k2[1, 1] = 1.0
    k2[2, 0] = k2[3, 1] = -1.0
    cfg = DenseModelConfig(["x"], ["y"], [2], [2], width=WIDTH, depth=2)
    params = dict(hidden_kernels=[k1], hidden_biases=[np.zeros(WIDTH, np.float32)], out_kernels=[k2],
                  out_biases=[np.zeros(2, np.float32)], in_mean=[mean], in_sigma=[std],
                  out_mean=[mean if denorm else np.zeros(2, np.float32)],
                  out_sigma=[std if denorm else np.ones(2, np.float32)])
    return DenseColumnModel(cfg, params)


def test_fit_is_the_reference_fit():
    from fv3net_amd import normalization

    mean, std = normalization.fit_mean_std(X)
    np.testing.assert_array_equal(mean, [0.5, 1.0])
    np.testing.assert_array_equal(std, [0.5, 1.0])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_oracle_kat(dtype):
    norm = dense_predict([X], _model(False).oracle_params(), dtype)[0]
    np.testing.assert_allclose(norm, NORM, rtol=1e-6)
    back = dense_predict([X], _model(True).oracle_params(), dtype)[0]
    np.testing.assert_allclose(back, X, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "bf16x3", "bf16x6"])
def test_kernel_kat(gpu, precision):
    import torch

    x = torch.from_numpy(X.T.copy()).cuda()  # [feature, sample]
    norm = _model(False).forward([x], precision=precision)[0].cpu().numpy().T
    np.testing.assert_allclose(norm, NORM, rtol=1e-6)
    back = _model(True).forward([x], precision=precision)[0].cpu().numpy().T
    np.testing.assert_allclose(back, X, rtol=1e-6, atol=1e-6)
