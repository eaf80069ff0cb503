"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package restates, in plain numpy / torch-autograd fp64, the reference's
hot path (AlexGisi/mpc-racing ``control/MPC.py`` NLP and its ``splines/``
inputs).  It is the *checker* for the HIP product in ``mpc-racing_amd/``:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product never imports, links or
executes anything under ``oracle/``.

Pinning status:
  * splines (``oracle.splines``): pinned against golden vectors produced by
    the reference's own ``splines/`` package (tests/golden/make_golden.py).
  * dynamics (``oracle.dynamics``): pinned against the values recorded from
    ``control/MPC.py`` in SURVEY.md §8(c); the blend law against the numpy
    models (golden G7 uses ``models/BlendedBicycleModel.py``).
  * NLP solution (``oracle.nlp``): the reference's solver (CasADi 3.6.5 /
    IPOPT, not vendored, not installable here) cannot run, so the NLP of
    ``control/MPC.py:30-161`` is restated and solved to a tight KKT tolerance
    by a dense primal-dual interior point method, cross-checked against
    scipy SLSQP.  Parity with IPOPT itself is UNPINNED.
"""
