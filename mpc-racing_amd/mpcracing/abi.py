"""ctypes mirror of ``include/mpcracing.h`` (the C ABI of libmpcracing.so)."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.abspath(os.path.join(HERE, "..", "csrc"))
PRODUCT_LIB = os.path.join(CSRC, "libmpcracing.so")
HOST_TWIN_LIB = os.path.join(CSRC, "libmpcracing_host.so")

ABI_VERSION = 102  # MR_ABI_VERSION of include/mpcracing.h
MR_MODEL = {"kin": 0, "dyn": 1, "blend": 2, "blend_pacejka": 3, "dyn_pacejka": 4}
MR_PREC = {"fp64": 0, "fp32": 1}
STATUS = {0: "solved", 1: "acceptable", 2: "max_iter", 3: "failed", 4: "infeasible"}

_I32 = ctypes.c_int32
_D = ctypes.c_double
_PD = ctypes.POINTER(ctypes.c_double)
_PI32 = ctypes.POINTER(ctypes.c_int32)


class MRConfig(ctypes.Structure):
    _fields_ = [(n, _I32) for n in ("N", "model", "precision", "lane_bounds", "max_batch", "device",
                                    "max_iter", "acceptable_iter")] + \
               [(n, _D) for n in ("Ts", "tol", "acceptable_tol",
                                  "lambda_s", "alpha_L", "min_steer", "max_steer", "min_throttle",
                                  "max_steer_delta", "min_steer_delta", "max_throttle_delta",
                                  "min_throttle_delta", "q_v_max", "v_max", "min_s_delta",
                                  "m", "Iz", "lf", "lr", "Cf", "Cr", "T_max", "r_wheel", "C_wheel", "R",
                                  "rho", "C_d", "A_f", "C_roll", "g", "max_steer_deg", "Vblendmin",
                                  "Vblendmax")] + [("dispatch_order", _I32)]


class MRInputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("state0", "s0", "cx", "cy", "max_error", "runtime", "u_init",
                                               "order_hint")]


class MROutputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("X", "U", "S", "eC", "eL", "status", "iters", "obj", "kkt",
                                               "trace")] + [("trace_instance", _I32), ("trace_cap", _I32),
                                                           ("lam_g", ctypes.c_void_p), ("timeline", ctypes.c_void_p),
                                                           ("constr_viol", ctypes.c_void_p)]


# every symbol declared in include/mpcracing.h (checked by tests/test_abi.py)
EXPORTS = ["mr_version", "mr_last_error", "mr_config_default", "mr_create", "mr_destroy", "mr_set_tyres",
           "mr_solve_batch", "mr_workspace_bytes_per_instance", "mr_eval_dynamics",
           "mr_track_create", "mr_track_destroy", "mr_track_eval", "mr_track_frame", "mr_track_error_sign",
           "mr_track_polyfit", "mr_track_polyfit_deg", "mr_track_lookup_error", "mr_track_projection", "mr_track_prep",
           "mr_spline_from_waypoints", "mr_track_lane_table", "mr_agent_sense", "mr_plant_step"]


def _bind_product(lib):
    lib.mr_version.restype = ctypes.c_int
    lib.mr_last_error.restype = ctypes.c_char_p
    lib.mr_config_default.argtypes = [ctypes.POINTER(MRConfig)]
    lib.mr_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(MRConfig)]
    lib.mr_destroy.argtypes = [ctypes.c_void_p]
    lib.mr_set_tyres.argtypes = [ctypes.c_void_p, _PD, _D, _PD, _D]
    lib.mr_solve_batch.argtypes = [ctypes.c_void_p, _I32, ctypes.POINTER(MRInputs), ctypes.POINTER(MROutputs),
                                   ctypes.c_void_p]
    lib.mr_eval_dynamics.argtypes = [ctypes.c_void_p, _I32] + [ctypes.c_void_p] * 7
    lib.mr_workspace_bytes_per_instance.argtypes = [ctypes.c_void_p]
    lib.mr_workspace_bytes_per_instance.restype = ctypes.c_int64
    V = ctypes.c_void_p
    lib.mr_track_create.argtypes = [ctypes.POINTER(V), _I32, _PD, _I32, _PD, _PD, _I32, _D, _PD, _PD, _I32]
    lib.mr_track_destroy.argtypes = [V]
    lib.mr_track_eval.argtypes = [V, _I32, V, V, V, V]
    lib.mr_track_frame.argtypes = [V, _I32, V, V, V, V, V, _D, V, V]
    lib.mr_track_error_sign.argtypes = [V, _I32, V, V, V, V, V]
    lib.mr_track_polyfit.argtypes = [V, _I32, V, V, V, V, V]
    lib.mr_track_polyfit_deg.argtypes = [V, _I32, V, V, _I32, V, V, V]
    lib.mr_track_lookup_error.argtypes = [V, _I32, V, V, V, V, V, V, V]
    lib.mr_track_projection.argtypes = [V, _I32, V, V, V, V, V, V, V, V]
    lib.mr_track_prep.argtypes = [V, _I32, V, V, V, V, _D, _D, _D, V, V, V, V, V, V]
    lib.mr_spline_from_waypoints.argtypes = [_PD, _PD, _I32, _I32, _PD, _PD, _PD, _PI32, _PD]
    lib.mr_track_lane_table.argtypes = [V, V, _I32, V, V, V, V]
    lib.mr_agent_sense.argtypes = [V, _I32, V, V, V, _D, _D, _D, V, V, V, V, V, V]
    lib.mr_plant_step.argtypes = [_I32, _I32, V, V, _D, V, V]
    return lib


_product = None


def load_product(path=None):
    """Load the gfx950 library. There is no fallback: a missing library is an error.
    MR_PRODUCT_LIB may name another build of the same source (developer A/B runs)."""
    global _product
    path = path or os.environ.get("MR_PRODUCT_LIB") or PRODUCT_LIB
    if _product is None:
        if not os.path.exists(path):
            raise RuntimeError(f"libmpcracing.so not built ({path}); run `python __graft_entry__.py build`")
        lib = _bind_product(ctypes.CDLL(path))
        if lib.mr_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: ABI version {lib.mr_version()}, this binding expects {ABI_VERSION} "
                               "(rebuild with `python __graft_entry__.py build`)")
        _product = lib
    return _product


def load_host_twin(path=HOST_TWIN_LIB):
    """TEST-ONLY host build of the same solver source (never used by the product path)."""
    lib = ctypes.CDLL(path)
    lib.mrh_config_default.argtypes = [ctypes.POINTER(MRConfig)]
    lib.mrh_solve_batch.argtypes = [ctypes.POINTER(MRConfig), _PD, _D, _PD, _D, ctypes.c_int,
                                    ctypes.POINTER(MRInputs), ctypes.POINTER(MROutputs), ctypes.c_int]
    lib.mrh_solve_batch_scalar.argtypes = lib.mrh_solve_batch.argtypes
    lib.mrh_eval_dynamics.argtypes = [ctypes.POINTER(MRConfig), _PD, _D, _PD, _D, _PD, _PD, _PD, _PD, _PD, _PD]
    lib.mrh_pacejka.argtypes = [_PD, _D, _D, ctypes.c_int, _PD]
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.mrh_track_blob_size.argtypes = [I, I]
    lib.mrh_track_build.argtypes = [V, I, V, V, I, V, V, I, V]
    lib.mrh_track_eval.argtypes = [V, I, _D, I, I, V, V, V]
    lib.mrh_track_frame.argtypes = [V, I, _D, I, I, V, V, V, V, V, _D, V]
    lib.mrh_track_sign.argtypes = [V, I, _D, I, I, V, V, V, V]
    lib.mrh_track_polyfit.argtypes = [V, I, _D, I, I, V, V, V, V]
    lib.mrh_track_polyfit_deg.argtypes = [V, I, _D, I, I, V, V, I, V, V]
    lib.mrh_track_lookup.argtypes = [V, I, _D, I, I, V, V, V, V, V, V]
    lib.mrh_track_projection.argtypes = [V, I, _D, I, I, V, V, V, V, V, V, V]
    lib.mrh_spline_from_waypoints.argtypes = [_PD, _PD, I, I, _PD, _PD, _PD, _PI32, _PD]
    lib.mrh_lane_table.argtypes = [V, I, _D, I, V, I, _D, I, V, V, V]
    lib.mrh_agent_sense.argtypes = [V, I, _D, I, I, V, V, V, _D, _D, _D, V, V, V, V, V]
    lib.mrh_plant_step.argtypes = [I, I, V, V, _D, V]
    return lib
