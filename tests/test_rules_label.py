"""``oracle.ipopt.PRODUCT`` is the rule set the kernel compiles, not a description of it.

Every IPOPT rule the product can switch at compile time is a macro default in csrc/mr_solver.h (shared by the
scalar solver and the gfx950 wave kernel, csrc/mr_wave.h).  The oracle's PRODUCT rule set is what the
fixtures built by tests/golden/make_solution_golden.py, make_dropin_golden.py and make_c3_sample_golden.py and
the live comparisons of test_duals / test_host_twin / test_cpu_baseline / test_ipopt_trajectory run; this test
reads the macro defaults back and requires PRODUCT to carry the same switches (round-5 ADVICE: PRODUCT kept
IPOPT's tiny-step rule while the kernel compiled it out).
"""
import os
import re

from oracle import ipopt

HERE = os.path.dirname(os.path.abspath(__file__))
SOLVER = os.path.join(HERE, "..", "mpc-racing_amd", "csrc", "mr_solver.h")

# macro -> the PRODUCT field it decides
RULE_MACROS = {
    "MR_TINY_STEP": "tiny_step",
    "MR_SOFT_RESTO": "soft_resto",
    "MR_RESTO_LS_MULT": "resto_ls_mult",
}


def _defaults():
    src = open(SOLVER).read()
    out = {}
    for m in RULE_MACROS:
        hit = re.search(r"#ifndef %s\s*\n#define %s (\d+)" % (m, m), src)
        assert hit, m
        out[m] = int(hit.group(1))
    return out


def test_product_rules_mirror_the_kernel_switches():
    d = _defaults()
    for m, field in RULE_MACROS.items():
        assert getattr(ipopt.PRODUCT, field) == bool(d[m]), (m, d[m], field, getattr(ipopt.PRODUCT, field))


def test_product_differs_from_ipopt_only_in_documented_rules():
    """The fields where PRODUCT leaves IPOPT's rules are exactly the deviations DESIGN.md §2 lists."""
    diff = {f for f in ipopt.Rules.__dataclass_fields__ if getattr(ipopt.PRODUCT, f) != getattr(ipopt.IPOPT, f)}
    assert diff <= {"tiny_step", "resto_ls_mult", "resto_soc", "resto_watchdog", "resto_relax_x0"}, diff
    assert "tiny_step" in diff
