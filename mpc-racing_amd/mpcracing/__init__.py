"""mpcracing -- MI355X-native batched racing-MPC solver (host side).

The reference's hot path (AlexGisi/mpc-racing ``control/MPC.py``: a CasADi Opti
NLP solved by IPOPT, one instance per call) is replaced by ``libmpcracing.so``:
one gfx950 thread per MPC instance runs a primal-dual interior-point solve with
Riccati-structured Newton steps.  This package holds the host side: the ctypes
binding (``abi``), batch assembly on device tensors (``batch``), track assets
and synthetic workloads (``track``, ``workload``).  The drop-in modules that
mirror the reference layout live beside it: ``control/``, ``models/``.
"""
__version__ = "0.1.0"
