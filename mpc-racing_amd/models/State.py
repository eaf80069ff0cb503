"""Vehicle state record (reference models/State.py:5-36)."""
from dataclasses import dataclass
import math


@dataclass
class State:
    x: float          # global X (m)
    y: float          # global Y (m)
    yaw: float        # heading (rad)
    v_x: float        # body-frame longitudinal speed (m/s)
    v_y: float        # body-frame lateral speed (m/s)
    yaw_dot: float    # yaw rate (rad/s)
    steer: float = None      # last steer command, None disables the stage-0 steer-rate row
    throttle: float = None   # last throttle command, None disables the stage-0 throttle-rate row

    def set_controls(self, throttle, steer):
        self.throttle = throttle
        self.steer = steer
        return self

    def as_state0_row(self):
        """The [x, y, yaw, v_x, v_y, yaw_dot, throttle, steer] column of mr_inputs.state0 (NaN = None)."""
        nan = math.nan
        return [float(self.x), float(self.y), float(self.yaw), float(self.v_x), float(self.v_y),
                float(self.yaw_dot), nan if self.throttle is None else float(self.throttle),
                nan if self.steer is None else float(self.steer)]
