"""Batched solve on the GPU through libmpcracing.so (PyTorch tensors for device storage only).

``BatchSolver`` is the batch API behind the drop-in ``control.MPC.MPC``: it
owns a solver handle (workspace sized for ``max_batch``) and solves B
independent instances per call.  Inputs/outputs follow the structure-of-arrays
layout of include/mpcracing.h.  There is no CPU fallback: without a GPU or
without the built library the constructor raises.
"""
import ctypes

import numpy as np
import torch

from . import abi

_IN_KEYS = ("state0", "s0", "cx", "cy", "max_error", "runtime", "u_init")


class BatchSolver:
    def __init__(self, N, model="dyn", precision="fp64", lane=False, Ts=0.05, max_batch=1, device=0, tol=None,
                 tyres=None, **overrides):
        if not torch.cuda.is_available():
            raise RuntimeError("mpcracing.BatchSolver needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = abi.load_product()
        c = abi.MRConfig()
        self.lib.mr_config_default(ctypes.byref(c))
        c.N = int(N)
        c.model = abi.MR_MODEL[model]
        c.precision = abi.MR_PREC[precision]
        c.lane_bounds = int(bool(lane))
        c.Ts = float(Ts)
        c.max_batch = int(max_batch)
        c.device = int(device)
        if tol is not None:
            c.tol = float(tol)
        elif precision == "fp32":
            # the reference's own IPOPT options (control/MPC.py:152-161): tol 1e-4, acceptable_tol 1e-2,
            # IPOPT's acceptable_iter 15 (the fp32 solve resolves the KKT error to 1e-4 through its fp64
            # multipliers, mr_wave.h eval_sweep; the acceptable exit catches the rare stalls)
            c.tol = 1e-4
            c.acceptable_tol = 1e-2
        for k, v in overrides.items():
            setattr(c, k, v)
        self.cfg = c
        self.device = torch.device("cuda", int(device))
        self.N = int(N)
        h = ctypes.c_void_p()
        self._check(self.lib.mr_create(ctypes.byref(h), ctypes.byref(c)))
        self.h = h
        if tyres is not None:
            (af, Fzf), (ar, Fzr) = tyres
            af = np.asarray(af, np.float64)
            ar = np.asarray(ar, np.float64)
            self._check(self.lib.mr_set_tyres(h, af.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), float(Fzf),
                                              ar.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), float(Fzr)))

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"libmpcracing error {rc}: {self.lib.mr_last_error().decode()}")

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.mr_destroy(h)
            self.h = None

    def to_device(self, batch):
        out = {}
        h = batch.get("order_hint")
        if h is not None:  # int32 [B] (dispatch_order 2), e.g. a previous solve's iters
            out["order_hint"] = (h if isinstance(h, torch.Tensor) else torch.from_numpy(np.asarray(h))).to(
                self.device, torch.int32).contiguous()
        for k in _IN_KEYS:
            v = batch.get(k)
            if v is None:
                out[k] = None
            elif isinstance(v, torch.Tensor):
                out[k] = v.to(self.device, torch.float64).contiguous()
            else:
                out[k] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(self.device)
        return out

    def alloc_outputs(self, B, duals=False):
        """Output tensors; ``duals`` adds ``lam_g`` [13N+9][B] (the reference's opti.lam_g, Opti row order)."""
        N, d = self.N, self.device
        f = dict(dtype=torch.float64, device=d)
        out = {"X": torch.empty((6, N + 1, B), **f), "U": torch.empty((2, N, B), **f),
               "S": torch.empty((N + 1, B), **f), "eC": torch.empty((N, B), **f), "eL": torch.empty((N, B), **f),
               "status": torch.empty(B, dtype=torch.int32, device=d),
               "iters": torch.empty(B, dtype=torch.int32, device=d),
               "obj": torch.empty(B, **f), "kkt": torch.empty(B, **f), "constr_viol": torch.empty(B, **f)}
        if duals:
            out["lam_g"] = torch.empty((13 * N + 9, B), **f)
        return out

    def launch(self, dev_in, out, stream=None, trace_instance=-1):
        """Enqueue one batched solve on ``stream`` (default: torch's current stream); no sync."""
        B = int(dev_in["s0"].shape[0])
        N = self.N
        shapes = {"state0": (8, B), "s0": (B,), "cx": (5, B), "cy": (5, B), "max_error": (B,), "runtime": (5, B),
                  "u_init": (2, N, B)}
        for k, shp in shapes.items():
            v = dev_in.get(k)
            if v is None:
                continue
            if tuple(v.shape) != shp or v.dtype != torch.float64 or not v.is_contiguous() or v.device != self.device:
                raise ValueError(f"input {k}: expected contiguous float64 {shp} on {self.device}, got "
                                 f"{tuple(v.shape)} {v.dtype} {v.device}")
        h = dev_in.get("order_hint")
        if h is not None and (tuple(h.shape) != (B,) or h.dtype != torch.int32 or not h.is_contiguous()
                              or h.device != self.device):
            raise ValueError(f"input order_hint: expected contiguous int32 ({B},) on {self.device}")
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        inp = abi.MRInputs(*[ptr(dev_in.get(k)) for k in _IN_KEYS + ("order_hint",)])
        tr = out.get("trace")
        o = abi.MROutputs(*[ptr(out.get(k)) for k in ("X", "U", "S", "eC", "eL", "status", "iters", "obj", "kkt",
                                                      "trace")], int(trace_instance),
                          int(tr.shape[0]) if tr is not None else 0, ptr(out.get("lam_g")),
                          ptr(out.get("timeline")), ptr(out.get("constr_viol")))
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._check(self.lib.mr_solve_batch(self.h, B, ctypes.byref(inp), ctypes.byref(o),
                                            ctypes.c_void_p(st.cuda_stream)))
        return out

    def solve(self, batch, stream=None, trace_instance=-1, trace_cap=0, duals=False):
        """Blocking solve of a host or device batch; returns device output tensors."""
        dev_in = self.to_device(batch)
        out = self.alloc_outputs(int(dev_in["s0"].shape[0]), duals=duals)
        if trace_cap:
            out["trace"] = torch.zeros((trace_cap, 8), dtype=torch.float64, device=self.device)
        self.launch(dev_in, out, stream, trace_instance)
        torch.cuda.synchronize(self.device)
        return out


def solver_for_config(name, max_batch, device=0, **kw):
    """BatchSolver configured as BASELINE config ``name`` (C1..C5)."""
    from .workload import CONFIGS, tyre_coeffs
    c = CONFIGS[name]
    tyres = tyre_coeffs(c["tyres"]) if c["tyres"] else None
    precision = kw.pop("precision", c["precision"])
    return BatchSolver(c["N"], c["model"], precision, c["lane"], c["Ts"], max_batch=max_batch,
                       device=device, tyres=tyres, **kw)
