"""``simulation/planner.py`` — the straight-line ego reference the hot path and the QP consume.

Reference: ``ReferenceTrajectoryPlanner.straight_line_trajectory`` (``simulation/planner.py:120-197``),
host NumPy as in the reference (it runs once per scenario, O(horizon)).  ``plan_trajectory``
(``:35-118``, a CVXPY goal-tracking QP that no caller of the hot path uses) is out of scope.
"""
from __future__ import annotations

import numpy as np



class ReferenceTrajectoryPlanner:
    def __init__(self, A, B, C, Q, R, horizon, dt):
        self.A = np.asarray(A, dtype=np.float64)
        self.B = np.asarray(B, dtype=np.float64)
        self.C = np.asarray(C, dtype=np.float64)
        self.Q = Q
        self.R = R
        self.horizon = horizon
        self.dt = dt
        self.n_states = self.A.shape[0]
        self.n_inputs = self.B.shape[1]
        self.n_outputs = self.C.shape[0]

    def straight_line_trajectory(self, start_pos, goal_pos, velocity=1.5):
        """(x_ref [H+1, nx], u_ref [H, nu], info): constant-speed line to the goal, then hold;
        inputs from ``u_t = pinv(B) (x_{t+1} - A x_t)`` (planner.py:187-190)."""
        start_pos = np.asarray(start_pos, dtype=np.float64)
        goal_pos = np.asarray(goal_pos, dtype=np.float64)
        direction = goal_pos - start_pos
        distance = np.linalg.norm(direction)
        H = self.horizon
        x_ref = np.zeros((H + 1, self.n_states))
        u_ref = np.zeros((H, self.n_inputs))
        if distance < 1e-10:
            x_ref[:, :2] = start_pos
            return x_ref, u_ref, {"status": "OPTIMAL", "distance": 0.0}
        direction = direction / distance
        time_to_goal = distance / velocity
        n_steps = int(time_to_goal / self.dt)
        x_ref[0, :2] = start_pos
        for t in range(1, H + 1):
            if t <= n_steps:
                x_ref[t, :2] = start_pos + (t / n_steps) * (goal_pos - start_pos)
                x_ref[t, 2:] = velocity * direction
            else:
                x_ref[t, :2] = goal_pos
        pinv_b = np.linalg.pinv(self.B)
        for t in range(H):
            u_ref[t] = pinv_b @ (x_ref[t + 1] - self.A @ x_ref[t])
        return x_ref, u_ref, {"status": "OPTIMAL", "distance": distance,
                              "time_to_goal": time_to_goal, "n_steps": n_steps}
