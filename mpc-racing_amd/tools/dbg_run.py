import os, sys
sys.path.insert(0, 'mpc-racing_amd'); sys.path.insert(0, 'tests')
import torch  # noqa: F401  (torch first: one HIP runtime in the process)
from mpcracing import abi
abi.load_product(os.path.join(abi.CSRC, 'libmpcracing_dbg.so'))
from mpcracing import workload as wl
from mpcracing.batch import BatchSolver
b = wl.make_batch('C4', limit=2)
s = BatchSolver(40, 'blend', 'fp64', max_batch=2, acceptable_iter=0, max_iter=1)
o = s.solve(b, trace_instance=0, trace_cap=200)
print(o['status'].cpu().numpy())
