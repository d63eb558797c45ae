"""CPU checks of the drop-in boundary: libppo.so loads, exports every function include/*.h declares,
and its struct layouts match the ctypes mirror.  No compute calls (no GPU here)."""
import ctypes as C
import os
import subprocess
import sys

import ppo_ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo.c_amd", "tools"))
from exports import declared_functions  # noqa: E402


def test_every_declared_function_is_exported(lib_built):
    decl = declared_functions()
    assert len(decl) >= 90
    out = subprocess.run(["nm", "-D", "--defined-only", ppo_ffi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [f"{h}:{n}" for h, n in decl if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    # and nothing beyond the header set leaks out (version script)
    extra = exported - {n for _, n in decl}
    assert not extra, f"exported but not declared: {sorted(extra)[:20]}"


def test_reference_api_surface_present(lib_built):
    """Every function of the reference headers (ppo.h, neural_network.h, …) is part of the ABI."""
    ref_names = """create_ppo free_ppo collect_trajectories compute_gae policy_loss_and_grad compute_gae_cuda
    policy_loss_and_grad_cuda train_ppo_epoch eval_ppo save_ppo load_ppo create_neural_network
    forward_propagation free_neural_network backward_propagation forward_propagation_cuda
    backward_propagation_cuda nn_write_weights_to_device nn_write_weights_to_host save_neural_network
    load_neural_network create_trajectory_buffer free_trajectory_buffer shuffle_buffer get_batch
    shuffle_buffer_cuda get_batch_cuda reset_buffer buffer_to_device buffer_to_host create_gaussian_policy
    free_gaussian_policy sample_action compute_log_prob log_prob_backwards compute_log_prob_cuda
    log_prob_backwards_cuda compute_entropy_cuda compute_entropy policy_to_host save_policy load_policy
    create_adam create_adam_from_nn free_adam adam_update create_adam_cuda create_adam_from_nn_cuda
    free_adam_cuda adam_update_cuda save_adam load_adam load_adam_from_nn mean_squared_error
    mean_squared_error_derivative mean_squared_error_cuda mean_squared_error_derivative_cuda mat_mul
    mat_mul_backwards mat_mul_cuda mat_mul_backwards_cuda ReLU ReLU_derivative ReLU_cuda
    ReLU_derivative_cuda build_activation_function build_activation_function_cuda create_simple_env
    create_gym_env openblas_set_num_threads""".split()
    for n in ref_names:
        assert hasattr(lib_built, n), n


def test_struct_layouts_match_ctypes(lib_built):
    sizes = (C.c_long * 7)()
    assert lib_built.ppo_struct_sizes(sizes, 7) == 7
    for s, cls in zip(sizes, ppo_ffi.STRUCTS):
        assert s == C.sizeof(cls), f"{cls.__name__}: C {s} vs ctypes {C.sizeof(cls)}"


def test_reference_main_compiles_unchanged_against_headers(tmp_path):
    """The reference's main.c (as shipped) compiles against include/ with no warnings (gcc and clang)."""
    main_c = "/root/reference/src/main.c"
    if not os.path.exists(main_c):      # the GPU box has no reference tree; the built bin/ppo_main travels
        assert os.path.exists(os.path.join(ROOT, "ppo.c_amd", "bin", "ppo_main"))
        return
    for cc in ("gcc", "/opt/rocm/llvm/bin/clang"):
        r = subprocess.run([cc, "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-c", main_c, "-o",
                            str(tmp_path / "main.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_no_gpu_means_no_device(lib_built):
    """Without a GPU the library reports 0 devices instead of silently computing on the CPU."""
    n = lib_built.ppo_device_count()
    assert n >= 0
