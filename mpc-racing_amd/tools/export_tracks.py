"""Export the reference's track assets as inert data files for the product.

Run here (where ``/root/reference`` exists); the GPU box only sees the output
``mpc-racing_amd/data/tracks/<track>.npz``.  Each file holds the raw waypoint
list of ``waypoints/<track>`` (track id dropped, exactly as
``splines/ParameterizedCenterline.py:95`` does), the two lane-boundary point
lists of ``lanes/<track>_{left,right}.csv`` and the lane-width table
``lanes/<track>_max_error.csv`` (columns ss, right, left).  No derived
quantity is stored: the spline is rebuilt by the product from the waypoints
(``mpcracing/track.py``), as the reference does at start-up.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from safe_pickle import load_waypoint_pickle  # noqa: E402

REF = "/root/reference"
TRACKS = ["shanghai_intl_circuit", "t1_triple", "t2_triple", "t3", "t4"]


def _csv(path):
    # pandas' default float parser (as the reference reads these files,
    # ParameterizedCenterline.py:17-25, ParameterizedLane.py:22-25) is not
    # round-trip exact; store the values exactly as the reference sees them.
    import pandas as pd
    df = pd.read_csv(path)
    return {h: df[h].to_numpy(dtype=np.float64).copy() for h in df.columns}


def main(out_dir=os.path.join(HERE, "..", "data", "tracks")):
    os.makedirs(out_dir, exist_ok=True)
    for t in TRACKS:
        wp = load_waypoint_pickle(os.path.join(REF, "waypoints", t))
        track_id = wp[0]
        pts = np.array(wp[1:], dtype=np.float64)
        left = _csv(os.path.join(REF, "lanes", f"{t}_left.csv"))
        right = _csv(os.path.join(REF, "lanes", f"{t}_right.csv"))
        err = _csv(os.path.join(REF, "lanes", f"{t}_max_error.csv"))
        np.savez_compressed(
            os.path.join(out_dir, f"{t}.npz"),
            track_id=np.int64(track_id), waypoints=pts,
            left_csv_x=left["x"], left_csv_y=left["y"],
            right_csv_x=right["x"], right_csv_y=right["y"],
            err_ss=err["ss"], err_right=err["right"], err_left=err["left"])
        print(t, pts.shape, len(err["ss"]))


if __name__ == "__main__":
    main()
