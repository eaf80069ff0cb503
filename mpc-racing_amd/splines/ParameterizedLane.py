"""Drop-in ``splines.ParameterizedLane`` (splines/ParameterizedLane.py:6-25): a lane boundary
line with the stateful progress window used by the offline lane-width table build."""
from splines.ParameterizedLine import ParameterizedLine


class ParameterizedLane(ParameterizedLine):
    def __init__(self):
        super().__init__()
        self.last_progress = None  # progress of the last projection

    def progress_bounds(self, step=0.5):
        if self.last_progress is None:
            return None
        return (self.last_progress - (2 * step), self.last_progress + (step * 6))

    def projection(self, X, Y, bounds=None):
        ret = super().projection(X, Y, bounds)
        self.last_progress = ret[0]
        return ret

    def from_file(self, fp):
        """lanes/<track>_{left,right}.csv with columns x, y."""
        import pandas as pd
        df = pd.read_csv(fp)
        self.from_waypoints(list(zip(df["x"], df["y"])))

    def from_xy(self, xy):
        """The same from an [n][2] array (the repo's exported track data)."""
        self.from_waypoints([tuple(p) for p in xy])
