"""ORACLE binding — test infrastructure only.

numpy wrappers around oracle/build/liboracle.so (the plain-C restatement of
the reference CPU path, see ref_cpu.h).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this module, and only as the checker.
"""
import ctypes as C
import glob
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_f32 = np.float32
_lib = None


class RefUpdateCfg(C.Structure):
    _fields_ = [("num_sizes", C.c_int), ("sizes_mu", C.c_int * 8), ("relu", C.c_int * 8), ("N", C.c_int),
                ("batch_size", C.c_int), ("n_epochs_policy", C.c_int), ("n_epochs_value", C.c_int),
                ("gamma", C.c_float), ("lambda_", C.c_float), ("epsilon", C.c_float), ("ent_coeff", C.c_float),
                ("lr_policy", C.c_float), ("lr_v", C.c_float), ("shuffle_mode", C.c_int), ("seed", C.c_uint64),
                ("max_value_steps", C.c_int), ("max_policy_steps", C.c_int)]


_FP = C.POINTER(C.c_float)


class RefUpdateState(C.Structure):
    _fields_ = [("mu_params", _FP), ("log_std", _FP), ("v_params", _FP),
                ("m_mu", _FP), ("v_mu", _FP), ("t_mu", C.c_int),
                ("m_v", _FP), ("v_v", _FP), ("t_v", C.c_int),
                ("m_ent", _FP), ("v_ent", _FP), ("t_ent", C.c_int),
                ("state", _FP), ("next_state", _FP), ("action", _FP), ("reward", _FP), ("logprob", _FP),
                ("terminated", C.POINTER(C.c_uint8)), ("truncated", C.POINTER(C.c_uint8)),
                ("advantage", _FP), ("adv_target", _FP),
                ("sum_v_loss", C.c_double), ("sum_policy_loss", C.c_double), ("n_v", C.c_long), ("n_p", C.c_long),
                ("adv_mean", C.c_float), ("adv_std", C.c_float),
                ("t_gae", C.c_double), ("t_value", C.c_double), ("t_policy", C.c_double)]


def openblas_path():
    try:
        import numpy
        cands = glob.glob(os.path.join(os.path.dirname(numpy.__file__), "..", "numpy.libs",
                                       "libscipy_openblas64_*.so"))
        return os.path.abspath(cands[0]) if cands else ""
    except Exception:
        return ""


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load(use_openblas=False):
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        lib.ref_mse.restype = C.c_float
        lib.ref_entropy.restype = C.c_float
        lib.ref_policy_loss_and_grad.restype = C.c_float
        lib.ref_mlp_num_params.restype = C.c_long
        lib.ref_feistel_index.restype = C.c_uint32
        lib.ref_feistel_index.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        lib.ref_feistel_perm.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
        lib.ref_blas_load.argtypes = [C.c_char_p]
        lib.ref_blas_name.restype = C.c_char_p
        lib.ref_adam_update.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long,
                                        C.POINTER(C.c_int), C.c_float, C.c_float, C.c_float]
        lib.ref_gae.argtypes = [C.c_void_p] * 5 + [C.c_int, C.c_float, C.c_float, C.c_void_p, C.c_void_p,
                                                   C.POINTER(C.c_float), C.POINTER(C.c_float)]
        lib.ref_policy_loss_and_grad.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_void_p, C.c_void_p,
                                                 C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_int]
        lib.ref_ppo_update.argtypes = [C.POINTER(RefUpdateCfg), C.POINTER(RefUpdateState)]
        lib.ref_relu.argtypes = [C.c_void_p, C.c_long]
        lib.ref_relu_derivative.argtypes = [C.c_void_p, C.c_void_p, C.c_long]
        _lib = lib
    if use_openblas:
        _lib.ref_blas_load(openblas_path().encode())
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _ints(xs):
    arr = (C.c_int * len(xs))()
    arr[:] = list(xs)
    return arr


# ---------------------------------------------------------------- ops
def mat_mul(x, W, b):
    lib = load()
    m, n = x.shape
    l = W.shape[0]
    out = np.empty((m, l), _f32)
    lib.ref_mat_mul(_p(out), _p(np.ascontiguousarray(x, _f32)), _p(np.ascontiguousarray(W, _f32)),
                    _p(np.ascontiguousarray(b, _f32)), m, n, l)
    return out


def mat_mul_backwards(g, x, W, gx0=None, gW0=None):
    """Accumulating (β=1) CPU semantics: returns gx0 + g·W, gW0 + gᵀ·x."""
    lib = load()
    m, l = g.shape
    n = x.shape[1]
    gx = np.zeros((m, n), _f32) if gx0 is None else np.array(gx0, _f32, copy=True)
    gW = np.zeros((l, n), _f32) if gW0 is None else np.array(gW0, _f32, copy=True)
    lib.ref_mat_mul_backwards(_p(gx), _p(gW), _p(np.ascontiguousarray(g, _f32)),
                              _p(np.ascontiguousarray(x, _f32)), _p(np.ascontiguousarray(W, _f32)), m, n, l)
    return gx, gW


def relu(x):
    y = np.array(x, _f32, copy=True)
    load().ref_relu(_p(y), y.size)
    return y


def relu_derivative(y, g):
    g2 = np.array(g, _f32, copy=True)
    load().ref_relu_derivative(_p(np.ascontiguousarray(y, _f32)), _p(g2), g2.size)
    return g2


def mse(y, t):
    y = np.ascontiguousarray(y, _f32).ravel()
    t = np.ascontiguousarray(t, _f32).ravel()
    lib = load()
    loss = lib.ref_mse(_p(y), _p(t), y.size, 1)
    g = np.empty_like(y)
    lib.ref_mse_derivative(_p(g), _p(y), _p(t), y.size, 1)
    return float(loss), g


# ---------------------------------------------------------------- MLP
def mlp_num_params(sizes):
    return int(load().ref_mlp_num_params(len(sizes), _ints(sizes)))


def mlp_init(sizes):
    p = np.empty(mlp_num_params(sizes), _f32)
    load().ref_mlp_init(len(sizes), _ints(sizes), _p(p))
    return p


def unpack(sizes, params):
    """flat packed params → [(W, b), ...]"""
    out, off = [], 0
    for i in range(len(sizes) - 1):
        n, l = sizes[i], sizes[i + 1]
        W = params[off:off + n * l].reshape(l, n)
        off += n * l
        b = params[off:off + l]
        off += l
        out.append((W, b))
    return out


def mlp_forward(sizes, relu_flags, params, x):
    m = x.shape[0]
    tot = sum(m * s for s in sizes[1:])
    acts = np.empty(tot, _f32)
    load().ref_mlp_forward(len(sizes), _ints(sizes), _ints(relu_flags), _p(np.ascontiguousarray(params, _f32)),
                           _p(np.ascontiguousarray(x, _f32)), m, _p(acts))
    return acts


def mlp_layer_outputs(sizes, acts, m):
    outs, off = [], 0
    for s in sizes[1:]:
        outs.append(acts[off:off + m * s].reshape(m, s))
        off += m * s
    return outs


def mlp_backward(sizes, relu_flags, params, x, acts, grad_out, want_gx=False):
    m = x.shape[0]
    grads = np.empty(mlp_num_params(sizes), _f32)
    gx = np.empty((m, sizes[0]), _f32) if want_gx else None
    load().ref_mlp_backward(len(sizes), _ints(sizes), _ints(relu_flags), _p(np.ascontiguousarray(params, _f32)),
                            _p(np.ascontiguousarray(x, _f32)), _p(acts), _p(np.ascontiguousarray(grad_out, _f32)),
                            m, _p(grads), _p(gx) if want_gx else None)
    return (grads, gx) if want_gx else grads


# ---------------------------------------------------------------- policy
def entropy(log_std):
    ls = np.ascontiguousarray(log_std, _f32)
    return float(load().ref_entropy(_p(ls), ls.size))


def log_prob(mu, log_std, action):
    m, A = mu.shape
    out = np.empty(m, _f32)
    load().ref_log_prob(_p(np.ascontiguousarray(mu, _f32)), _p(np.ascontiguousarray(log_std, _f32)),
                        _p(np.ascontiguousarray(action, _f32)), m, A, _p(out))
    return out


def log_prob_backwards(mu, log_std, action, grad_in):
    m, A = mu.shape
    gmu = np.empty((m, A), _f32)
    gls = np.empty(A, _f32)
    load().ref_log_prob_backwards(_p(np.ascontiguousarray(mu, _f32)), _p(np.ascontiguousarray(log_std, _f32)),
                                  _p(np.ascontiguousarray(action, _f32)), _p(np.ascontiguousarray(grad_in, _f32)),
                                  m, A, _p(gmu), _p(gls))
    return gmu, gls


def policy_loss_and_grad(adv, lp, old_lp, entropy_val, ent_coeff, epsilon):
    m = adv.size
    g = np.empty(m, _f32)
    ge = C.c_float(0)
    loss = load().ref_policy_loss_and_grad(_p(g), C.byref(ge), _p(np.ascontiguousarray(adv, _f32)),
                                           _p(np.ascontiguousarray(lp, _f32)),
                                           _p(np.ascontiguousarray(old_lp, _f32)), entropy_val, ent_coeff,
                                           epsilon, m)
    return float(loss), g, float(ge.value)


# ---------------------------------------------------------------- GAE / buffer / Adam
def gae(v, v_next, reward, term, trunc, gamma, lam):
    n = v.size
    adv = np.empty(n, _f32)
    tgt = np.empty(n, _f32)
    mean, std = C.c_float(0), C.c_float(0)
    load().ref_gae(_p(np.ascontiguousarray(v, _f32)), _p(np.ascontiguousarray(v_next, _f32)),
                   _p(np.ascontiguousarray(reward, _f32)), _p(np.ascontiguousarray(term, np.uint8)),
                   _p(np.ascontiguousarray(trunc, np.uint8)), n, gamma, lam, _p(adv), _p(tgt), C.byref(mean),
                   C.byref(std))
    return adv, tgt, float(mean.value), float(std.value)


def shuffle(n):
    perm = np.empty(n, np.int32)
    load().ref_shuffle(_p(perm), n)
    return perm


def feistel_perm(n, key):
    perm = np.empty(n, np.int32)
    load().ref_feistel_perm(_p(perm), n, key)
    return perm


def adam_update(params, grads, m, v, t, lr, beta1=0.9, beta2=0.999):
    """In-place on params/m/v (float32 arrays); returns the new time step."""
    ts = C.c_int(t)
    load().ref_adam_update(_p(params), _p(np.ascontiguousarray(grads, _f32)), _p(m), _p(v), params.size,
                           C.byref(ts), beta1, beta2, lr)
    return ts.value


def libc():
    return C.CDLL("libc.so.6")


def srand(seed):
    libc().srand(C.c_uint(seed))
