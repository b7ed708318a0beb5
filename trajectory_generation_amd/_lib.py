"""ctypes binding of libtrajmpc.so (the C ABI declared in include/trajmpc.h).

The library is built in-tree (trajectory_generation_amd/libtrajmpc.so, see csrc/Makefile).
There is no CPU fallback: if the library or a GPU is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# TRAJMPC_LIB: an alternative build of the same library (kernel-variant experiments, tools/)
LIB_PATH = os.environ.get("TRAJMPC_LIB") or os.path.join(_HERE, "libtrajmpc.so")
CSRC = os.path.join(_HERE, "csrc")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "trajmpc.h")
HEADERS = [HEADER, os.path.join(os.path.dirname(_HERE), "include", "trajknet.h")]

TRAJ_OK, TRAJ_E_ARG, TRAJ_E_UNSUPPORTED, TRAJ_E_LAUNCH, TRAJ_E_HANDOFF = 0, -1, -2, -3, -4
MAX_N = 40            # hot kernels, every entry point (include/trajmpc.h TRAJ_MAX_N)
MAX_N_SPLIT = 64      # the row-split kernel for SPLIT_MIN_N <= N <= MAX_N_SPLIT (TRAJ_MAX_N_SPLIT)
SPLIT_MIN_N = 21      # TRAJ_SPLIT_MIN_N
MAX_N_LONG = 256      # step / QP entry points on the long-horizon kernel without state bounds (TRAJ_MAX_N_LONG)
MAX_N_GENERAL = 1024  # step / QP entry points on the general solver (TRAJ_MAX_N_GENERAL)

STATUS_STRINGS = {
    0: "optimal",
    1: "optimal_inaccurate",
    2: "user_limit",
    3: "infeasible",
    4: "infeasible_inaccurate",
    5: "unbounded",
    6: "Solver Error: SolverError",
}

_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int)
_V = C.c_void_p


class VehicleParams(C.Structure):
    """traj_vehicle_params  (MPC/mpc_6stati.py:9-19)."""
    _fields_ = [(k, C.c_double) for k in (
        "Cm1", "Cm2", "Cr0", "Cr2", "Br", "Cr", "Dr", "Bf", "Cf", "Df", "m", "Iz", "lf", "lr", "g",
        "maxAlpha", "vx_zero")]


class MpcConfig(C.Structure):
    """traj_mpc_config  (mpc_step kwargs, MPC/mpc_6stati.py:120-143, + solver settings)."""
    _fields_ = [
        ("N", C.c_int), ("Ts", C.c_double),
        ("q_c", C.c_double), ("q_phi", C.c_double), ("q_vx", C.c_double),
        ("R", C.c_double * 4), ("Rd", C.c_double * 4),
        ("u_lo", C.c_double * 2), ("u_hi", C.c_double * 2),
        ("du_lo", C.c_double * 2), ("du_hi", C.c_double * 2),
        ("has_x_lo", C.c_int), ("has_x_hi", C.c_int),
        ("x_lo", C.c_double * 6), ("x_hi", C.c_double * 6),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double),
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double), ("delta", C.c_double),
        ("max_iter", C.c_int), ("check_interval", C.c_int), ("scaling_iters", C.c_int),
        ("polish", C.c_int), ("polish_refine_iter", C.c_int), ("adaptive_rho", C.c_int),
        ("adaptive_rho_tol", C.c_double),
        ("polish_mode", C.c_int), ("polish_max_pass", C.c_int), ("cert_tol", C.c_double),
        ("polish_max_rounds", C.c_int), ("warm_start", C.c_int),
    ]


class KnetLimits(C.Structure):
    """traj_knet_limits (state clamp limits of vehicle_model.py:54-57,125-131)."""
    _fields_ = [(k, C.c_float) for k in (
        "x_min", "x_max", "y_min", "y_max", "phi_min", "phi_max", "vx_min", "vx_max", "vy_min", "vy_max",
        "omega_min", "omega_max")]


class KnetNet(C.Structure):
    """traj_knet_net (device pointers to a KalmanNetNN's weights, include/trajknet.h)."""
    _fields_ = [(k, C.c_int) for k in ("m", "n", "hidden", "d_fc5", "d_fc1", "d_fc7", "d_fc3")] + [
        (k, C.c_void_p) for k in (
            "fc5_w", "fc5_b", "gru_q_wih", "gru_q_bih", "gru_q_whh", "gru_q_bhh", "gru_sigma_wih", "gru_sigma_bih",
            "gru_sigma_whh", "gru_sigma_bhh", "fc1_w", "fc1_b", "fc7_w", "fc7_b", "gru_s_wih", "gru_s_bih",
            "gru_s_whh", "gru_s_bhh", "fc3_w", "fc3_b", "fc4_w", "fc4_b", "innov_logit")] + [
        ("d_fc2h", C.c_int)] + [(k, C.c_void_p) for k in ("fc2a_w", "fc2a_b", "fc2b_w", "fc2b_b")]


class Paths(C.Structure):
    """traj_paths (closed-loop reference geometry per trajectory)."""
    _fields_ = [("kmax", C.c_int), ("kind", _V), ("pc", _V), ("nk", _V), ("xk", _V), ("coef", _V)]


# name -> (restype, argtypes)
_SIGS = {
    "traj_abi_version": (C.c_int, []),
    "traj_status_string": (C.c_char_p, [C.c_int]),
    "traj_error_string": (C.c_char_p, [C.c_int]),
    "traj_default_params": (C.c_int, [C.POINTER(VehicleParams)]),
    "traj_default_config": (C.c_int, [C.POINTER(MpcConfig), C.c_int, C.c_double]),
    "traj_tire_forces_batch": (C.c_int, [C.POINTER(VehicleParams), C.c_int, _V, _V, _V, _V]),
    "traj_f_cont_batch": (C.c_int, [C.POINTER(VehicleParams), C.c_int, _V, _V, _V, _V]),
    "traj_numerical_jacobian_batch": (C.c_int, [C.POINTER(VehicleParams), C.c_int, _V, _V, C.c_double,
                                                C.c_double, _V, _V, _V, _V]),
    "traj_linearize_discretize_batch": (C.c_int, [C.POINTER(VehicleParams), C.c_int, C.c_double, _V, _V, _V, _V,
                                                  _V, _V]),
    "traj_lateral_error_batch": (C.c_int, [C.c_int, _V, _V, _V, _V, _V, _V, _V]),
    "traj_mpc_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "traj_mpc_sb_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "traj_closed_loop_workspace_bytes": (C.c_size_t, [C.POINTER(MpcConfig), C.c_int]),
    "traj_mpc_step_batch": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(MpcConfig), C.c_int, _V, _V, _V, _V,
                                      _V, _V, _V, _V, _V, _V, _V, _V, C.c_size_t, _V]),
    "traj_mpc_qp_batch": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(MpcConfig), C.c_int, _V, _V, _V, _V, _V,
                                    _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, C.c_size_t, _V]),
    "traj_ref_window_batch": (C.c_int, [C.POINTER(Paths), C.c_int, C.c_int, C.c_double, _V, _V, _V, _V]),
    "traj_debug_set_stamps": (C.c_int, [_V]),
    "traj_debug_kernel_timing": (C.c_int, [C.c_int]),
    "traj_debug_fused_grid": (C.c_int, [C.c_int]),
    "traj_debug_spin_limit": (C.c_int, [C.c_int]),
    "traj_debug_queue_lead": (C.c_int, [C.c_int, C.c_int]),
    "traj_debug_run_ahead": (C.c_int, [C.c_int]),
    "traj_debug_fused_waves": (C.c_int, [C.c_int]),
    "traj_debug_step_linearize": (C.c_int, [C.c_int]),
    "traj_debug_split_max_n": (C.c_int, [C.c_int]),
    "traj_debug_split_min_n": (C.c_int, [C.c_int]),
    "traj_debug_set_item_stamps": (C.c_int, [_V]),
    "traj_closed_loop_check": (C.c_int, [_V, C.c_size_t, C.c_int, C.c_int, _V]),
    "traj_dataset_write_csv": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_double, _V, _V, _V, _V,
                                         C.c_int]),
    "traj_dataset_csv_rows": (C.c_longlong, [C.c_char_p, _V]),
    "traj_dataset_read_csv": (C.c_int, [C.c_char_p, C.c_longlong, C.c_int, _V, C.c_int]),
    "traj_debug_kernel_times": (C.c_int, [_V, _V]),
    "traj_knet_prior_f32": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(KnetLimits), C.c_float, C.c_int,
                                      _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "traj_knet_gru_gates_f32": (C.c_int, [C.c_int, C.c_int, _V, _V, _V, _V, _V]),
    "traj_knet_update_f32": (C.c_int, [C.c_int, _V, _V, _V, _V, _V, _V]),
    "traj_knet_packed_bytes": (C.c_size_t, [C.POINTER(KnetNet)]),
    "traj_knet_pack_f32": (C.c_int, [C.POINTER(KnetNet), _V, C.c_size_t, _V]),
    "traj_knet_front_f32": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(KnetLimits), C.c_float,
                                      C.POINTER(KnetNet), _V, C.c_int, _V, _V, C.c_int, C.c_int, _V, C.c_int,
                                      C.c_int, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "traj_knet_fc2_workspace_bytes": (C.c_size_t, [C.POINTER(KnetNet), C.c_int]),
    "traj_knet_fc2_f32": (C.c_int, [C.POINTER(KnetNet), C.c_int, _V, _V, C.c_size_t, _V]),
    "traj_knet_set_fc2_mode": (C.c_int, [C.c_int]),
    "traj_knet_back_f32": (C.c_int, [C.POINTER(KnetNet), _V, C.c_int, _V, _V, _V, _V, _V, _V, _V, C.c_int,
                                     C.c_int, _V, _V]),
    "traj_knet_back_front_f32": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(KnetLimits), C.c_float,
                                           C.POINTER(KnetNet), _V, C.c_int, _V, _V, C.c_int, C.c_int, _V, C.c_int,
                                           C.c_int, _V, C.c_int, C.c_int, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V,
                                           _V, _V, _V, _V]),
    "traj_knet_rollout_windows": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "traj_knet_rollout_eval_f32": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(KnetLimits), C.c_float, C.c_int,
                                             C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _V, C.c_int, C.c_int, C.c_int,
                                             _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "traj_ekf_run_f64": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(KnetLimits), C.c_double, C.c_int, C.c_int,
                                   _V, _V, _V, _V, _V, _V, _V, _V]),
    "traj_closed_loop_step": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(MpcConfig), C.POINTER(Paths), C.c_int,
                                        _V, _V, _V, C.c_int, C.c_int, _V, _V, _V, _V, _V, C.c_size_t, _V]),
    "traj_closed_loop_run": (C.c_int, [C.POINTER(VehicleParams), C.POINTER(MpcConfig), C.POINTER(Paths), C.c_int,
                                        _V, _V, _V, C.c_int, C.c_int, C.c_int, _V, _V, _V, _V, _V, C.c_size_t, _V]),
}

_lib = None


def build(jobs: int = 8) -> str:
    """Compile libtrajmpc.so for gfx950 with hipcc (csrc/Makefile)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True)
    return LIB_PATH


def lib():
    """Load the HIP library (raises if it is missing -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                               "or __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("TRAJMPC_LIB") and name.startswith("traj_debug_") and not hasattr(L, name):
                continue   # an older variant build (experiments) may lack a newer diagnostic entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.traj_abi_version() != 4:
            raise RuntimeError("libtrajmpc ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != TRAJ_OK:
        msg = lib().traj_error_string(rc).decode()
        if rc == TRAJ_E_UNSUPPORTED:
            raise NotImplementedError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed: {msg} ({rc})")


def default_params() -> VehicleParams:
    p = VehicleParams()
    check(lib().traj_default_params(C.byref(p)), "traj_default_params")
    return p


def default_config(N: int, Ts: float) -> MpcConfig:
    c = MpcConfig()
    check(lib().traj_default_config(C.byref(c), int(N), float(Ts)), "traj_default_config")
    return c


def exported_symbols() -> list[str]:
    return list(_SIGS)
