"""Scenario data of ``config/scenarios.py:11-68`` (the active block): start/goal/obstacle motion."""
import numpy as np

_SCENARIOS = {
    "head_on": dict(ego_start=(-4.0, 0.0), ego_goal=(4.0, 0.0), obstacle_start=(4.0, 0.0),
                    obstacle_direction=(-1.0, 0.0), description="Head-on collision scenario"),
    "overtaking": dict(ego_start=(-4.0, 0.0), ego_goal=(4.0, 0.0), obstacle_start=(-2.0, 0.0),
                       obstacle_direction=(1.0, 0.0), obstacle_speed=0.7,
                       description="Overtaking scenario"),
    "intersection": dict(ego_start=(-4.0, 0.0), ego_goal=(4.0, 0.0), obstacle_start=(0.0, 4.0),
                         obstacle_direction=(0.0, -1.0), obstacle_speed=1.5,
                         description="Intersection crossing scenario"),
    "multi_obstacle": dict(ego_start=(-2.0, -1.0), ego_goal=(4.0, 0.0), obstacles=[
        dict(start=(0.0, 2.0), direction=(0.0, -0.5), speed=0.8),
        dict(start=(-3.0, 0.5), direction=(0.7, 0.0), speed=0.6),
        dict(start=(1.5, -2.0), direction=(-0.2, 0.5), speed=0.7)],
        description="Multiple obstacle scenario"),
}


def get_scenario_config(scenario_name):
    """Fresh dict with NumPy arrays, as the reference returns (``config/scenarios.py:11``)."""
    if scenario_name not in _SCENARIOS:
        raise ValueError(f"Unknown scenario: {scenario_name}")
    src = _SCENARIOS[scenario_name]
    cfg = {}
    for k, v in src.items():
        if k == "obstacles":
            cfg[k] = [{kk: (np.array(vv) if isinstance(vv, tuple) else vv) for kk, vv in ob.items()}
                      for ob in v]
        else:
            cfg[k] = np.array(v) if isinstance(v, tuple) else v
    return cfg
