"""Shared helpers for the parity tests (numpy <-> libppo device memory, tolerances)."""
import ctypes as C

import numpy as np

import ppo_ffi

F32 = np.float32


def dev(lib, arr):
    return ppo_ffi.DeviceArray.from_numpy(lib, np.ascontiguousarray(arr))


def empty(lib, count, dtype=F32):
    return ppo_ffi.DeviceArray(lib, int(count) * np.dtype(dtype).itemsize)


def gemm_tol(ref, K):
    """Stated fp32 GEMM tolerance: 1e-4·‖ref‖∞ + 1e-6 for K ≤ 1024, growing as √K beyond."""
    scale = max(1.0, (K / 1024.0) ** 0.5)
    return 1e-4 * scale * float(np.abs(ref).max(initial=0.0)) + 1e-6


def assert_gemm_close(got, ref, K, what=""):
    err = float(np.abs(got - ref).max(initial=0.0))
    tol = gemm_tol(ref, K)
    assert err <= tol, f"{what}: max |err| {err:.3g} > tol {tol:.3g} (K={K})"


def assert_rel_close(got, ref, rtol, atol, what=""):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    bad = np.abs(got - ref) > atol + rtol * np.abs(ref)
    assert not bad.any(), (f"{what}: {int(bad.sum())}/{bad.size} outside rtol={rtol} atol={atol}; "
                           f"worst {float(np.abs(got - ref).max()):.3g}")


def nn_params_packed(lib, nn_ptr):
    """Packed [W0,b0,W1,b1,...] (reference order) read back from a libppo NeuralNetwork's HBM buffer."""
    nn = nn_ptr.contents
    out = []
    for i in range(nn.num_layers - 1):
        ly = nn.layers[i]
        nw = ly.input_size * ly.output_size
        out.append(ppo_ffi.d2h(lib, ly.d_weights, F32, nw))
        out.append(ppo_ffi.d2h(lib, ly.d_biases, F32, ly.output_size))
    return np.concatenate(out)


def nn_grads_packed(lib, nn_ptr):
    nn = nn_ptr.contents
    out = []
    for i in range(nn.num_layers - 1):
        ly = nn.layers[i]
        nw = ly.input_size * ly.output_size
        out.append(ppo_ffi.d2h(lib, ly.d_grad_weights, F32, nw))
        out.append(ppo_ffi.d2h(lib, ly.d_grad_biases, F32, ly.output_size))
    return np.concatenate(out)


def nn_set_params_packed(lib, nn_ptr, params):
    nn = nn_ptr.contents
    off = 0
    for i in range(nn.num_layers - 1):
        ly = nn.layers[i]
        nw = ly.input_size * ly.output_size
        ppo_ffi.h2d(lib, ly.d_weights, params[off:off + nw].astype(F32))
        off += nw
        ppo_ffi.h2d(lib, ly.d_biases, params[off:off + ly.output_size].astype(F32))
        off += ly.output_size
    assert off == params.size


def c_float_ptr(x):
    return C.cast(x, C.c_void_p)
