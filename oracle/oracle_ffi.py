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
                ("max_value_steps", C.c_int), ("max_policy_steps", C.c_int), ("capacity", C.c_int)]


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


def blas_mode(mode):
    """Chaos-floor perturbation of the oracle's products (ref_cpu.c): 0 = the oracle proper,
    1 = split-K halves, 2 = double-precision products rounded once to fp32.  Needs OpenBLAS."""
    if load(use_openblas=True).ref_blas_mode(int(mode)) != 0:
        raise RuntimeError(f"oracle: blas mode {mode} unavailable")


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


def ppo_update(sizes, relu_flags, mu_params, log_std, v_params, buf, *, batch_size, n_epochs_policy=4,
               n_epochs_value=10, gamma=0.99, lam=0.95, epsilon=0.2, ent_coeff=0.0, lr_policy=3e-4, lr_v=3e-4,
               shuffle_mode=0, seed=0, max_value_steps=-1, max_policy_steps=-1, adam=None, capacity=0):
    """One reference CPU update (ppo.cu:395-443 without the rollout) on copies of the inputs.

    buf: dict of numpy arrays state, next_state, action, reward, logprob, terminated, truncated — the
    `limit` filled rows of the buffer; capacity (> limit) gives a partly filled buffer's minibatch count.
    adam: optional dict with m/v/t for 'mu', 'v', 'ent' (fresh zeros otherwise).
    Returns a dict with the updated parameters, Adam state, advantages and loss sums.
    """
    lib = load()
    N = buf["reward"].size
    cfg = RefUpdateCfg()
    cfg.num_sizes = len(sizes)
    for i, s in enumerate(sizes):
        cfg.sizes_mu[i] = s
    for i, r in enumerate(relu_flags):
        cfg.relu[i] = r
    cfg.N, cfg.batch_size = N, batch_size
    cfg.n_epochs_policy, cfg.n_epochs_value = n_epochs_policy, n_epochs_value
    cfg.gamma, cfg.lambda_, cfg.epsilon, cfg.ent_coeff = gamma, lam, epsilon, ent_coeff
    cfg.lr_policy, cfg.lr_v = lr_policy, lr_v
    cfg.shuffle_mode, cfg.seed = shuffle_mode, seed
    cfg.max_value_steps, cfg.max_policy_steps = max_value_steps, max_policy_steps
    cfg.capacity = capacity
    out = {"mu": np.array(mu_params, _f32, copy=True), "log_std": np.array(log_std, _f32, copy=True),
           "v": np.array(v_params, _f32, copy=True), "advantage": np.zeros(N, _f32),
           "adv_target": np.zeros(N, _f32)}
    A = sizes[-1]
    ad = adam or {}
    for k, n in (("mu", out["mu"].size), ("v", out["v"].size), ("ent", A)):
        st = ad.get(k, {})
        out["m_" + k] = np.array(st.get("m", np.zeros(n, _f32)), _f32, copy=True)
        out["v_" + k] = np.array(st.get("v", np.zeros(n, _f32)), _f32, copy=True)
    keep = {k: np.ascontiguousarray(buf[k], _f32) for k in ("state", "next_state", "action", "reward", "logprob")}
    keep["terminated"] = np.ascontiguousarray(buf["terminated"], np.uint8)
    keep["truncated"] = np.ascontiguousarray(buf["truncated"], np.uint8)

    def fp(a):
        return a.ctypes.data_as(C.POINTER(C.c_float))

    st = RefUpdateState()
    st.mu_params, st.log_std, st.v_params = fp(out["mu"]), fp(out["log_std"]), fp(out["v"])
    st.m_mu, st.v_mu, st.t_mu = fp(out["m_mu"]), fp(out["v_mu"]), ad.get("mu", {}).get("t", 0)
    st.m_v, st.v_v, st.t_v = fp(out["m_v"]), fp(out["v_v"]), ad.get("v", {}).get("t", 0)
    st.m_ent, st.v_ent, st.t_ent = fp(out["m_ent"]), fp(out["v_ent"]), ad.get("ent", {}).get("t", 0)
    st.state, st.next_state, st.action = fp(keep["state"]), fp(keep["next_state"]), fp(keep["action"])
    st.reward, st.logprob = fp(keep["reward"]), fp(keep["logprob"])
    st.terminated = keep["terminated"].ctypes.data_as(C.POINTER(C.c_uint8))
    st.truncated = keep["truncated"].ctypes.data_as(C.POINTER(C.c_uint8))
    st.advantage, st.adv_target = fp(out["advantage"]), fp(out["adv_target"])
    lib.ref_ppo_update(C.byref(cfg), C.byref(st))
    out.update(t_mu=st.t_mu, t_v=st.t_v, t_ent=st.t_ent, sum_v_loss=st.sum_v_loss,
               sum_policy_loss=st.sum_policy_loss, n_v=st.n_v, n_p=st.n_p, adv_mean=st.adv_mean,
               adv_std=st.adv_std, t_gae=st.t_gae, t_value=st.t_value, t_policy=st.t_policy)
    return out


def libc():
    return C.CDLL("libc.so.6")


def srand(seed):
    libc().srand(C.c_uint(seed))


def save_ppo_bytes(hyper, S, A, capacity, log_std, mu_sizes, mu_acts, mu_params, v_sizes, v_acts, v_params,
                   adams):
    """The reference checkpoint writer, restated byte for byte (test infrastructure only).

    ppo.cu:585-611 save_ppo: lambda, epsilon, ent_coeff, lr_policy, lr_V (f32), state_size,
    action_size, capacity (i32); then save_policy (policy.cu:207-211: log_std[A] f32, then μ's
    save_neural_network), save_neural_network(V) (neural_network.cu:283-300: num_layers,
    output_size, per activation (strlen+1, chars incl. NUL), per layer (in, out, W[out·in], b[out])),
    and save_adam for adam_policy, adam_V, adam_entropy (adam.cu:172-189: size, time_step, beta1,
    beta2, num_layers, m[size], v[size]).  Everything native-endian (x86: little).
    hyper = (lambda, epsilon, ent_coeff, lr_policy, lr_V); adams = three dicts with keys
    size, t, b1, b2, n, m, v (m/v packed in tensor order).
    """
    import struct

    out = bytearray()
    out += struct.pack("<5f", *hyper)
    out += struct.pack("<3i", S, A, capacity)

    def nn(sizes, acts, params):
        b = bytearray(struct.pack("<2i", len(sizes), sizes[-1]))
        for a in acts:
            raw = a.encode() + b"\0"
            b += struct.pack("<i", len(raw)) + raw
        off = 0
        for i in range(len(sizes) - 1):
            n_in, n_out = sizes[i], sizes[i + 1]
            b += struct.pack("<2i", n_in, n_out)
            b += np.asarray(params[off:off + n_in * n_out + n_out], "<f4").tobytes()
            off += n_in * n_out + n_out
        assert off == len(params)
        return b

    out += np.asarray(log_std, "<f4").tobytes()
    out += nn(mu_sizes, mu_acts, mu_params)
    out += nn(v_sizes, v_acts, v_params)
    for ad in adams:
        out += struct.pack("<2i2fi", ad["size"], ad["t"], ad["b1"], ad["b2"], ad["n"])
        out += np.asarray(ad["m"], "<f4").tobytes() + np.asarray(ad["v"], "<f4").tobytes()
    return bytes(out)


def splitmix64(z):
    """libppo's key derivation (host/ppo.c splitmix64), for predicting device-shuffle permutations."""
    M = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def gaussian_noise(n):
    """ref_gaussian_noise (policy.cu:46-65, D3: every element filled); consumes libc rand()."""
    out = np.empty(n, _f32)
    load().ref_gaussian_noise(_p(out), n)
    return out
