"""Constants of ``config/parameters.py:11-33`` (the active, non-commented block)."""
ALPHA = 0.2            # CVaR level
DELTA = 0.1            # risk bound
EPSILON = 0.15         # Wasserstein radius
ROBOT_RADIUS = 0.3
DT = 0.2
HORIZON = 30
Q_WEIGHT = 2.0
R_WEIGHT = 1.0
SIM_TIME = 30.0
NUM_SAMPLES = 20
OBSTACLE_RADIUS = 0.3
OBSTACLE_SPEED = 1.0
NUM_MC_RUNS = 300
