"""ctypes binding of libppo's C ABI (include/*.h) for tests and bench.py.

This is the same binding a Python maintainer of the reference would write
(see INTEGRATION.md): plain pointers and sizes, the reference's structs
mirrored field by field.  It imports no torch and never falls back to CPU
math: if lib/libppo.so is missing, load() raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libppo.so")

c_float_p = C.POINTER(C.c_float)
c_int_p = C.POINTER(C.c_int)
c_bool_p = C.POINTER(C.c_bool)
c_long_p = C.POINTER(C.c_long)
VOIDFN = C.c_void_p


class ActivationFunction(C.Structure):
    _fields_ = [("activation", C.c_void_p), ("activation_derivative", C.c_void_p)]


class Layer(C.Structure):
    _fields_ = [(n, c_float_p) for n in ("weights", "biases", "grad_weights", "grad_biases", "input",
                                          "d_weights", "d_biases", "d_grad_weights", "d_grad_biases",
                                          "d_input", "d_grad_x")] + [
        ("activation_function", C.POINTER(ActivationFunction)),
        ("d_activation_function", C.POINTER(ActivationFunction)),
        ("input_size", C.c_int), ("output_size", C.c_int)]


class NeuralNetwork(C.Structure):
    _fields_ = [("layers", C.POINTER(Layer)), ("num_layers", C.c_int), ("output_size", C.c_int),
                ("cache_m_forward", C.c_int), ("cache_m_backward", C.c_int),
                ("output", c_float_p), ("d_output", c_float_p), ("activation_functions", C.POINTER(C.c_char_p)),
                ("cublas_handle", C.c_void_p),
                ("d_params", c_float_p), ("d_grads", c_float_p), ("num_params", C.c_long),
                ("num_params_packed", C.c_long), ("param_offset", c_long_p), ("bias_offset", c_long_p),
                ("act_cap_m", C.c_int), ("grad_cap_m", C.c_int), ("host_cap_m", C.c_int),
                ("extra_floats", C.c_long), ("d_x0", c_float_p), ("d_act_bits", C.POINTER(C.c_uint)),
                ("bits_m", C.c_int), ("dtype", C.c_int), ("x0_dtype", C.c_int), ("d_w16", C.c_void_p),
                ("d_tiny_wt", c_float_p), ("tiny_wt_cap", C.c_long),
                ("h_sync", c_float_p), ("dev_version", C.c_long),
                ("host_version", C.c_long), ("host_version_w", C.c_long),
                ("d_fold_ws", c_float_p), ("fold_ws_cap", C.c_long)]


class GaussianPolicy(C.Structure):
    _fields_ = [("mu", C.POINTER(NeuralNetwork)), ("log_std", c_float_p), ("log_std_grad", c_float_p),
                ("d_log_std", c_float_p), ("d_log_std_grad", c_float_p), ("state_size", C.c_int),
                ("action_size", C.c_int), ("input_action", c_float_p), ("d_input_action", c_float_p)]


_BUF_PTRS = ["state_p", "action_p", "next_state_p", "reward_p", "logprob_p", "advantage_p", "adv_target_p",
             "terminated_p", "truncated_p"]


class TrajectoryBuffer(C.Structure):
    pass


TrajectoryBuffer._fields_ = (
    [(n, c_bool_p if "terminated" in n or "truncated" in n else c_float_p) for n in _BUF_PTRS]
    + [("h_" + n, c_bool_p if "terminated" in n or "truncated" in n else c_float_p) for n in _BUF_PTRS]
    + [("d_" + n, c_bool_p if "terminated" in n or "truncated" in n else c_float_p) for n in _BUF_PTRS]
    + [("random_idx", c_int_p), ("state_size", C.c_int), ("action_size", C.c_int), ("capacity", C.c_int),
       ("idx", C.c_int), ("full", C.c_bool)]
    + [(n, VOIDFN) for n in ("state", "action", "next_state", "reward", "logprob", "advantage", "adv_target",
                             "terminated", "truncated")]
    + [("h_random_idx", c_int_p), ("on_device", C.c_int), ("random_idx_is_device", C.c_int)])


class Adam(C.Structure):
    _fields_ = [("weights", C.POINTER(c_float_p)), ("grad_weights", C.POINTER(c_float_p)), ("lengths", c_int_p),
                ("m", c_float_p), ("v", c_float_p), ("beta1", C.c_float), ("beta2", C.c_float),
                ("time_step", C.c_int), ("size", C.c_int), ("num_layers", C.c_int),
                ("on_device", C.c_int), ("flat", C.c_int), ("grad_scale", C.c_float), ("span", C.c_long)]


class PPO(C.Structure):
    _fields_ = [("buffer", C.POINTER(TrajectoryBuffer)), ("policy", C.POINTER(GaussianPolicy)),
                ("V", C.POINTER(NeuralNetwork)), ("adam_policy", C.POINTER(Adam)), ("adam_V", C.POINTER(Adam)),
                ("adam_entropy", C.POINTER(Adam)), ("lambda_", C.c_float), ("epsilon", C.c_float),
                ("ent_coeff", C.c_float), ("lr_policy", C.c_float), ("lr_V", C.c_float), ("use_cuda", C.c_bool),
                ("dev", C.c_void_p)]


class Env(C.Structure):
    _fields_ = [("free_env", VOIDFN), ("reset_env", VOIDFN), ("step_env", VOIDFN), ("state_size", C.c_int),
                ("action_size", C.c_int), ("horizon", C.c_int), ("gamma", C.c_float)]


STRUCTS = [Layer, NeuralNetwork, GaussianPolicy, TrajectoryBuffer, Adam, PPO, Env]

# name: (restype, argtypes)
_P = C.c_void_p
_F = c_float_p
_SIGS = {
    # runtime / ext
    "ppo_device_count": (C.c_int, []),
    "ppo_set_device": (C.c_int, [C.c_int]),
    "ppo_last_error": (C.c_char_p, []),
    "ppo_synchronize": (None, []),
    "ppo_gemm_tune": (C.c_int, [C.c_int, C.c_int]),
    "ppo_gemm16_tune": (C.c_int, [C.c_int]),
    "ppo_gemm_flags": (C.c_int, [C.c_int]),
    "ppo_bench_gemm16": (C.c_double, [C.c_int] * 7),
    "ppo_gemm_f32_engine": (C.c_int, [C.c_int]),
    "ppo_gemm16_dma": (C.c_int, [C.c_int]),
    "ppo_gemm16_tn_width": (C.c_int, [C.c_int]),
    "ppo_gemm_x3_tune": (C.c_int, [C.c_int, C.c_int]),
    "ppo_bench_gemm_x3": (C.c_double, [C.c_int] * 7),
    "ppo_x3_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "ppo_g16_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "ppo_set_compute_dtype": (C.c_int, [_P, C.c_int]),
    "ppo_rollout_device": (None, [_P, C.c_int, C.c_int, C.c_int, C.c_ulonglong]),
    "nn_set_compute_dtype": (C.c_int, [_P, C.c_int]),
    "ppo_bench_gemm": (C.c_double, [C.c_int] * 6),
    "ppo_bench_streams": (C.c_double, [C.c_int] * 4),
    "ppo_build_info": (C.c_char_p, []),
    "ppo_struct_sizes": (C.c_int, [c_long_p, C.c_int]),
    "ppo_dev_alloc": (_P, [C.c_size_t]),
    "ppo_dev_free": (None, [_P]),
    "ppo_h2d": (None, [_P, _P, C.c_size_t]),
    "ppo_d2h": (None, [_P, _P, C.c_size_t]),
    "ppo_d2d": (None, [_P, _P, C.c_size_t]),
    "ppo_dev_memset": (None, [_P, C.c_int, C.c_size_t]),
    "ppo_comm_unique_id": (C.c_int, [C.c_char_p, C.c_int]),
    "ppo_comm_init": (C.c_int, [C.c_int, C.c_int, C.c_char_p]),
    "ppo_comm_rank": (C.c_int, []),
    "ppo_comm_world": (C.c_int, []),
    "ppo_comm_finalize": (None, []),
    "ppo_comm_allreduce_f32": (None, [_P, C.c_long]),
    "ppo_welford_combine": (None, [_P, C.c_int, _P]),
    "ppo_comm_loopback_peers": (C.c_int, [_P, _P, C.c_int]),
    "ppo_comm_loopback_peer_grads": (C.c_int, [_P, _P, C.c_long]),
    "ppo_comm_loopback_clear": (None, []),
    "ppo_comm_loopback_peer_hash": (C.c_int, [_P, C.c_int]),
    "ppo_comm_mode": (C.c_char_p, []),
    "ppo_comm_check_replicas": (C.c_int, [_P]),
    "ppo_param_hash": (C.c_ulonglong, [_P]),
    "ppo_clear_error": (None, []),
    "ppo_nn_input_rows": (C.c_int, [_P, _P, C.c_int]),
    "ppo_gae_state": (C.c_long, [_P, _P, _P, C.c_long]),
    "ppo_comm_barrier": (None, []),
    "ppo_comm_max_f64": (C.c_double, [C.c_double]),
    "ppo_update": (None, [_P, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_ulonglong]),
    "ppo_read_stats": (None, [_P, C.POINTER(C.c_double), C.c_int]),
    "ppo_reset_stats": (None, [_P]),
    "ppo_set_step_limit": (None, [_P, C.c_long, C.c_long]),
    "ppo_sample_action_device": (None, [_P, _P, _P, _P, C.c_int, C.c_ulonglong, C.c_ulonglong]),
    "ppo_fill_synthetic": (None, [_P, C.c_int, C.c_int, C.c_ulonglong, C.c_float]),
    "ppo_prof_enable": (None, [C.c_int]),
    "ppo_prof_reset": (None, []),
    "ppo_prof_kernel_events": (None, [C.c_int]),
    "ppo_prof_shapes": (C.c_int, [C.POINTER(C.c_longlong), C.POINTER(C.c_double), c_long_p, C.POINTER(C.c_double),
                                  C.c_int]),
    "ppo_prof_read": (None, [C.POINTER(C.c_double), C.POINTER(C.c_double), c_long_p]),
    "ppo_prof_counts": (None, [c_long_p]),
    "ppo_prof_shape_issued": (C.c_int, [C.POINTER(C.c_longlong), c_long_p, C.c_int]),
    "ppo_prof_issued_work": (None, [C.POINTER(C.c_double)]),
    # mat_mul.h
    "mat_mul": (None, [_P, _P, _P, _P, C.c_int, C.c_int, C.c_int]),
    "mat_mul_backwards": (None, [_P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int]),
    "mat_mul_cuda": (None, [_P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int]),
    "mat_mul_backwards_cuda": (None, [_P, _P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int]),
    # activation / loss
    "ReLU": (None, [_P, C.c_int, C.c_int]),
    "ReLU_derivative": (None, [_P, _P, C.c_int, C.c_int]),
    "ReLU_cuda": (None, [_P, C.c_int, C.c_int]),
    "ReLU_derivative_cuda": (None, [_P, _P, C.c_int, C.c_int]),
    "mean_squared_error": (C.c_float, [_P, _P, C.c_int, C.c_int]),
    "mean_squared_error_derivative": (None, [_P, _P, _P, C.c_int, C.c_int]),
    "mean_squared_error_cuda": (C.c_float, [_P, _P, C.c_int, C.c_int]),
    "mean_squared_error_derivative_cuda": (None, [_P, _P, _P, C.c_int, C.c_int]),
    # neural network
    "create_neural_network": (C.POINTER(NeuralNetwork), [c_int_p, C.POINTER(C.c_char_p), C.c_int]),
    "free_neural_network": (None, [C.POINTER(NeuralNetwork)]),
    "forward_propagation": (None, [C.POINTER(NeuralNetwork), _P, C.c_int]),
    "backward_propagation": (None, [C.POINTER(NeuralNetwork), _P, C.c_int]),
    "forward_propagation_cuda": (None, [C.POINTER(NeuralNetwork), _P, C.c_int]),
    "backward_propagation_cuda": (None, [C.POINTER(NeuralNetwork), _P, C.c_int]),
    "nn_write_weights_to_device": (None, [C.POINTER(NeuralNetwork)]),
    "nn_write_weights_to_host": (None, [C.POINTER(NeuralNetwork)]),
    # policy
    "create_gaussian_policy": (C.POINTER(GaussianPolicy), [c_int_p, C.POINTER(C.c_char_p), C.c_int, C.c_float]),
    "free_gaussian_policy": (None, [C.POINTER(GaussianPolicy)]),
    "sample_action": (None, [C.POINTER(GaussianPolicy), _P, _P, _P, C.c_int]),
    "compute_log_prob": (None, [C.POINTER(GaussianPolicy), _P, _P, _P, C.c_int]),
    "log_prob_backwards": (None, [C.POINTER(GaussianPolicy), _P, _P, _P, C.c_int]),
    "compute_log_prob_cuda": (None, [C.POINTER(GaussianPolicy), _P, _P, _P, C.c_int]),
    "log_prob_backwards_cuda": (None, [C.POINTER(GaussianPolicy), _P, _P, _P, C.c_int]),
    "compute_entropy": (C.c_float, [C.POINTER(GaussianPolicy)]),
    "compute_entropy_cuda": (C.c_float, [C.POINTER(GaussianPolicy)]),
    "policy_to_host": (None, [C.POINTER(GaussianPolicy)]),
    # adam
    "create_adam_cuda": (C.POINTER(Adam), [C.POINTER(_P), C.POINTER(_P), c_int_p, C.c_int, C.c_int, C.c_float,
                                          C.c_float]),
    "create_adam_from_nn_cuda": (C.POINTER(Adam), [C.POINTER(NeuralNetwork), C.c_float, C.c_float]),
    "adam_update_cuda": (None, [C.POINTER(Adam), C.c_float]),
    "free_adam_cuda": (None, [C.POINTER(Adam)]),
    # buffer
    "create_trajectory_buffer": (C.POINTER(TrajectoryBuffer), [C.c_int, C.c_int, C.c_int]),
    "free_trajectory_buffer": (None, [C.POINTER(TrajectoryBuffer), C.c_bool]),
    "shuffle_buffer": (None, [C.POINTER(TrajectoryBuffer)]),
    "shuffle_buffer_cuda": (None, [C.POINTER(TrajectoryBuffer)]),
    "get_batch": (None, [C.POINTER(TrajectoryBuffer), C.c_int, C.c_int, _P, _P, _P, _P, _P]),
    "get_batch_cuda": (None, [C.POINTER(TrajectoryBuffer), C.c_int, C.c_int, _P, _P, _P, _P, _P]),
    "buffer_to_device": (None, [C.POINTER(TrajectoryBuffer)]),
    "buffer_to_host": (None, [C.POINTER(TrajectoryBuffer)]),
    "reset_buffer": (None, [C.POINTER(TrajectoryBuffer)]),
    # ppo
    "create_ppo": (C.POINTER(PPO), [C.POINTER(C.c_char_p), c_int_p, C.c_int, C.c_int, C.c_float, C.c_float,
                                    C.c_float, C.c_float, C.c_float, C.c_float, C.c_bool]),
    "free_ppo": (None, [C.POINTER(PPO)]),
    "compute_gae": (None, [C.POINTER(NeuralNetwork), C.POINTER(TrajectoryBuffer), C.c_float, C.c_float]),
    "compute_gae_cuda": (None, [C.POINTER(NeuralNetwork), C.POINTER(TrajectoryBuffer), C.c_float, C.c_float,
                                C.c_int]),
    "policy_loss_and_grad": (C.c_float, [_P, _F, _P, _P, _P, C.c_float, C.c_float, C.c_float, C.c_int]),
    "policy_loss_and_grad_cuda": (C.c_float, [_P, _F, _P, _P, _P, C.c_float, C.c_float, C.c_float, C.c_int]),
    "train_ppo_epoch": (None, [C.POINTER(PPO), C.POINTER(Env), C.c_int, C.c_int, C.c_int, C.c_int]),
    "eval_ppo": (None, [C.POINTER(PPO), C.POINTER(Env), C.c_int]),
    "save_ppo": (None, [C.POINTER(PPO), C.c_char_p]),
    "load_ppo": (C.POINTER(PPO), [C.c_char_p, C.c_bool]),
    "create_simple_env": (C.POINTER(Env), [C.c_int, C.c_int]),
    "create_gym_env": (C.POINTER(Env), [C.c_int, C.c_int]),
}

_lib = None


def load(path=None):
    """Load libppo.so (PPO_LIB overrides the path: diagnostic variants built by tools/build_variant.sh).

    In a process that also uses torch, `import torch` BEFORE calling load(): libppo then binds to the
    HIP runtime torch already mapped (same soname, libamdhip64.so.7) and the process holds one runtime.
    """
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("PPO_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"libppo.so not built at {path}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def c_strings(items):
    arr = (C.c_char_p * len(items))()
    arr[:] = [s.encode() for s in items]
    return arr


def c_ints(items):
    arr = (C.c_int * len(items))()
    arr[:] = list(items)
    return arr


class DeviceArray:
    """A float32/int32/uint8 array in HBM allocated through libppo (no torch)."""

    def __init__(self, lib, nbytes):
        self.lib = lib
        self.nbytes = max(int(nbytes), 4)
        self.ptr = lib.ppo_dev_alloc(self.nbytes)

    @classmethod
    def from_numpy(cls, lib, arr):
        import numpy as np
        arr = np.ascontiguousarray(arr)
        d = cls(lib, arr.nbytes)
        if arr.nbytes:
            lib.ppo_h2d(d.ptr, arr.ctypes.data, arr.nbytes)
        return d

    def to_numpy(self, dtype, count):
        import numpy as np
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            self.lib.ppo_d2h(out.ctypes.data, self.ptr, out.nbytes)
        return out

    def free(self):
        if self.ptr:
            self.lib.ppo_dev_free(self.ptr)
            self.ptr = None


def d2h(lib, ptr, dtype, count):
    import numpy as np
    out = np.empty(count, dtype=dtype)
    if out.nbytes:
        lib.ppo_d2h(out.ctypes.data, C.cast(ptr, C.c_void_p), out.nbytes)
    return out


def h2d(lib, ptr, arr):
    import numpy as np
    arr = np.ascontiguousarray(arr)
    if arr.nbytes:
        lib.ppo_h2d(C.cast(ptr, C.c_void_p), arr.ctypes.data, arr.nbytes)
