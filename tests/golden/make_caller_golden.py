"""Golden fixtures for the rows around the solve (build container only; needs /root/reference).

Writes ``tests/golden/callers_golden.json``:

  G4r   lane-table row keys read by ``lookup_error`` (splines/ParameterizedCenterline.py:61-80):
        the reference's ``lane_error_table.loc`` is wrapped in a recording proxy, so the first /
        last row read and the rows of the window minimum come from the reference's own loop
        (row index = 2 * key, the table's 0.5 m grid).  arg = the first row at which the side that
        ``min(right_min, left_min)`` returns reached its minimum (strict ``<`` updates).
  TS    ``TrackSegments(centerline, n_cp, v_max, d_f, d_r, m).bounds`` (splines/TrackSegments.py:7-35)
        for Shanghai (its ``__main__`` arguments) and t4.
  LOG   ``Logger.member_names``, one ``log_str`` row and the key order / value types of the
        ``pickle_mpc_res`` dict (Logger.py:5-50), with ``pickle.dump`` intercepted (nothing is
        written or unpickled).
  IMP   every ``splines.* / models.* / control.*`` import made by the reference's drop-in consumers
        (agent.py, GA/*.py, script/test_mpc.py), extracted from their source with ``ast``.
"""
import ast
import json
import os
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


class _LocRecorder:
    def __init__(self, df):
        self.df, self.keys = df, []

    @property
    def loc(self):
        rec = self

        class _L:
            def __getitem__(self, k):
                rec.keys.append(float(k))
                return rec.df.loc[k]
        return _L()


def _imports():
    out = {}
    files = ["agent.py", "GA/pdGA.py", "GA/mpcGA.py", "script/test_mpc.py"]
    for fn in files:
        tree = ast.parse(open(os.path.join(REF, fn)).read())
        mods = []
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and node.module and node.module.split(".")[0] in (
                    "splines", "models", "control"):
                mods.append({"module": node.module, "names": [a.name for a in node.names]})
            elif isinstance(node, ast.Import):
                for a in node.names:
                    if a.name.split(".")[0] in ("splines", "models", "control"):
                        mods.append({"module": a.name, "names": []})
        out[fn] = mods
    return out


def main():
    if not os.path.isdir(REF):
        raise SystemExit("make_caller_golden.py needs /root/reference (build container only)")
    sys.path.insert(0, HERE)
    from make_golden import _build_centerline
    os.chdir(REF)
    sys.path.insert(0, REF)
    res = {}
    # G4r
    g4 = {}
    for ti, track in enumerate(["shanghai_intl_circuit", "t1_triple", "t4"]):
        cl = _build_centerline(track)
        rec = _LocRecorder(cl.lane_error_table)
        cl.lane_error_table = rec
        rng = np.random.default_rng(3100 + ti)
        s = np.concatenate([rng.uniform(0.0, cl.length - 0.01, 60), [0.25, 0.75, 2.5, cl.length - 30.0]])
        la = np.concatenate([rng.choice([20.0, 45.0, 45.25, 75.0, 125.0, 175.0], 60), [45.0, 45.25, 75.0, 45.0]])
        rows = []
        for a, b in zip(s, la):
            rec.keys = []
            try:
                err = float(cl.lookup_error(a, b))
            except KeyError:
                rows.append({"s": float(a), "la": float(b), "err": None, "row_lo": -1, "row_hi": -1, "row_arg": -1})
                continue
            keys = rec.keys
            left = [float(rec.df.loc[k]["left"]) for k in keys]
            right = [float(rec.df.loc[k]["right"]) for k in keys]
            lm, rm, al, ar = 10000.0, 10000.0, -1, -1
            for j, k in enumerate(keys):
                if left[j] < lm:
                    lm, al = left[j], int(round(2 * k))
                if right[j] < rm:
                    rm, ar = right[j], int(round(2 * k))
            arg = al if lm < rm else ar
            assert min(rm, lm) == err
            rows.append({"s": float(a), "la": float(b), "err": err, "row_lo": int(round(2 * keys[0])),
                         "row_hi": int(round(2 * keys[-1])), "row_arg": arg, "n_rows_read": len(keys)})
        g4[track] = rows
    res["G4r"] = g4
    # TS
    from splines.TrackSegments import TrackSegments
    ts = {}
    for track, args in [("shanghai_intl_circuit", (10, 30, 1500, 1500, 250)), ("t4", (5, 30, 1500, 1500, 250))]:
        cl = _build_centerline(track)
        seg = TrackSegments(cl, *args)
        ts[track] = {"args": list(args), "bounds": [float(b) for b in seg.bounds], "lap_time": float(seg.lap_time)}
    res["TS"] = ts
    # LOG
    import Logger as LG
    captured = {}

    class _Agent:
        pass
    ag = _Agent()
    for i, k in enumerate(LG.member_names):
        setattr(ag, k, i + 0.5)
    ag.steps, ag.start_control_at = 60, 50
    ag.predicted_states, ag.last_controls = ["state"], [(0.1, 0.2)]
    ag.mean_ts, ag.mpc_time, ag.s_hat, ag.e_hat_c, ag.e_hat_l = 0.05, 0.01, np.zeros(3), [0.0], [0.0]
    orig_dump = LG.pickle.dump
    LG.pickle.dump = lambda obj, f, protocol=None: captured.update(obj=obj, protocol=protocol)
    lg = LG.Logger.__new__(LG.Logger)
    lg.mpc_fp = "/tmp/mr_caller_golden_mpc"
    os.makedirs(lg.mpc_fp, exist_ok=True)
    try:
        lg.pickle_mpc_res(ag)
    finally:
        LG.pickle.dump = orig_dump
    res["LOG"] = {"member_names": list(LG.member_names), "log_str": lg.log_str(ag),
                  "pickle_keys": list(captured["obj"].keys()),
                  "pickle_types": {k: type(v).__name__ for k, v in captured["obj"].items()},
                  "pickle_protocol": captured["protocol"]}
    # IMP
    res["IMP"] = _imports()
    with open(os.path.join(HERE, "callers_golden.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", os.path.join(HERE, "callers_golden.json"))


if __name__ == "__main__":
    main()
