"""MPC weights and bounds, same names and defaults as the reference.

Reference: control/ControllerParameters.py:3-32 (values from Costa et al., p. 8).
``FixedControllerParameters`` become mr_config fields of the solver handle;
``RuntimeControllerParameters`` are per-instance inputs ([5][B] runtime array).
Quirk kept: the upper throttle bound of the NLP is the CLASS attribute
``RuntimeControllerParameters.d_max`` (control/MPC.py:50), not the instance value.
"""
from dataclasses import dataclass


@dataclass
class FixedControllerParameters:
    lambda_s: float = 300          # progress reward at the horizon end
    alpha_L: float = 500           # lag-error weight
    min_steer: float = -0.9
    max_steer: float = 0.9
    min_throttle: float = -1.0
    max_steer_delta: float = 0.2
    min_steer_delta: float = -0.2
    max_throttle_delta: float = 2.0
    min_throttle_delta: float = -0.4
    q_v_max: float = 2             # soft speed-limit exponent rate
    v_max: float = 50
    Ts: float = 0.05               # default step when the caller passes Ts=None
    N: int = 30                    # default horizon when the caller passes N=None
    lookahead_distance: float = 30 * 0.05 * 50
    max_iter: int = 500


@dataclass
class RuntimeControllerParameters:
    alpha_c: float = 1000          # contouring-error weight
    d_max: float = 0.85            # max throttle (read as a class attribute by the NLP)
    q_v_y: float = 50              # lateral-velocity weight
    n: int = 2                     # exponent of the contouring error
    beta_delta: float = 5000       # steering-rate weight

    def as_runtime_row(self):
        """The [alpha_c, d_max, q_v_y, n, beta_delta] column of mr_inputs.runtime,
        with d_max taken from the class attribute as control/MPC.py:50 does."""
        return [float(self.alpha_c), float(RuntimeControllerParameters.d_max), float(self.q_v_y),
                float(self.n), float(self.beta_delta)]
