"""The C ABI: the product library exports exactly what include/mpcracing.h declares
(no compute call needs a GPU here), and the ctypes mirror matches the header."""
import ctypes
import os
import re
import subprocess

import pytest

from mpcracing import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mpcracing.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(mr_\w+)\s*\(", txt, flags=re.M)))


def test_header_declarations_match_mirror():
    assert declared_functions() == sorted(abi.EXPORTS)


@pytest.mark.skipif(not os.path.exists(abi.PRODUCT_LIB), reason="libmpcracing.so not built")
def test_product_library_exports_every_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.PRODUCT_LIB], capture_output=True, text=True,
                         check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for name in declared_functions():
        assert name in syms, name


@pytest.mark.skipif(not os.path.exists(abi.PRODUCT_LIB), reason="libmpcracing.so not built")
def test_config_default_without_gpu():
    lib = ctypes.CDLL(abi.PRODUCT_LIB)
    c = abi.MRConfig()
    lib.mr_config_default.argtypes = [ctypes.POINTER(abi.MRConfig)]
    assert lib.mr_config_default(ctypes.byref(c)) == 0
    # FixedControllerParameters / VehicleParameters defaults of the reference
    assert (c.N, c.max_iter, c.Ts, c.lambda_s, c.alpha_L, c.v_max) == (30, 500, 0.05, 300, 500, 50)
    assert c.C_wheel == 2 * 3.14 * 0.37 and c.max_steer_deg == 70.0 and c.min_s_delta == 0.1


def test_struct_layout_matches_header():
    # the C compiler's view of the struct sizes equals the ctypes mirror
    src = ('#include "%s"\n#include <stdio.h>\n#include <stddef.h>\nint main(){printf("%%zu %%zu %%zu %%zu\\n",'
           'sizeof(mr_config), sizeof(mr_inputs), sizeof(mr_outputs), offsetof(mr_config, Vblendmax));}' % HEADER)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "t.c"), "w").write(src)
        subprocess.run(["gcc", "-o", os.path.join(d, "t"), os.path.join(d, "t.c")], check=True)
        got = subprocess.run([os.path.join(d, "t")], capture_output=True, text=True, check=True).stdout.split()
    assert [int(v) for v in got] == [ctypes.sizeof(abi.MRConfig), ctypes.sizeof(abi.MRInputs),
                                     ctypes.sizeof(abi.MROutputs), abi.MRConfig.Vblendmax.offset]
