"""manipulator (3-DoF planar) system config (reference: conf_manipulator.py).

State (q0, q1, q2, q̇0, q̇1, q̇2, t); Pinocchio model from urdf/planar_manipulator_3dof.urdf
(revolute-Z links, gravity normal to the plane so nle is Coriolis/centrifugal only). Uses the
PiecewiseConstantDecay learning-rate schedule (conf_manipulator.py:51-72)."""
import math
import numpy as np
from ._common import finalize
from ..robots import builtin_model

system_id = 'manipulator'
UPDATE_LOOPS = np.arange(1000, 50000, 3000)
NUPDATES = 380000
NSTEPS = 100
BATCH_SIZE = 64
TD_DIV = 2
save_interval = 15000
plot_flag = 0
LR_SCHEDULE = 1
prioritized_replay_eps = 1e-2
fresh_factor = 0.95

XC1, YC1, A1, B1 = -2.0, 0.0, 6, 10
XC2, YC2, A2, B2 = 3.0, 4.0, 12, 4
XC3, YC3, A3, B3 = 3.0, -4.0, 12, 4
obs_param = np.array([XC1, YC1, XC2, YC2, XC3, YC3, A1, B1, A2, B2, A3, B3])
w_d, w_u, w_peak, w_ob, w_v = 100, 1, 5e5, 5e6, 1e4
cost_weights_running = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, w_u])
cost_weights_terminal = np.array([w_d, w_peak, w_v, w_ob, w_ob, w_ob, 0])
alpha, alpha2 = 50, 50
x_des, y_des = -20.0, 0.0
TARGET_STATE = np.array([x_des, y_des])

URDF_FILENAME = "planar_manipulator_3dof.urdf"
robot = builtin_model("planar_manipulator_3dof")
nq = robot.nq
nv = robot.nv
nx = nq + nv
na = robot.na
dt = 0.05
tau_coulomb_max = 0 * np.ones(robot.na)
q_init, v_init = np.array([math.pi, math.pi, math.pi]), np.zeros(robot.nv)
x_base, y_base = -7.0, 0.0
nb_state = robot.nq + robot.nv + 1
_pi, _p4 = math.pi, math.pi / 4
x_min = np.array([-np.inf] * 6 + [0])
x_init_min = np.array([-_pi, -_pi, -_pi, -_p4, -_p4, -_p4, 0])
x_max = np.array([np.inf] * 7)
x_init_max = np.array([_pi, _pi, _pi, _p4, _p4, _p4, (NSTEPS - 1) * dt])
state_norm_arr = np.array([15, 15, 15, 10, 10, 10, int(NSTEPS * dt)])
init_states_sim = [np.array(list(q) + [0.0, 0.0, 0.0, 0.0]) for q in (
    (_pi / 4, -_pi / 8, -_pi / 8), (-_pi / 4, _pi / 8, _pi / 8), (_pi / 2, 0.0, 0.0),
    (-_pi / 2, 0.0, 0.0), (3 * _pi / 4, 0.0, 0.0), (-3 * _pi / 4, 0.0, 0.0), (_pi / 4, 0.0, 0.0),
    (-_pi / 4, 0.0, 0.0), (_pi, 0.0, 0.0), (-1.55135003, 2.93707696, -1.3025857),
    (1.55135003, -2.93707696, 1.3025857), (-1.31811607, 2.63623214, -1.31811607),
    (-0.98843209, 1.97686418, -0.98843209))]
tau_lower_bound, tau_upper_bound = -200, 200
u_min = tau_lower_bound * np.ones(robot.na)
u_max = tau_upper_bound * np.ones(robot.na)
fig_ax_lim = np.array([[-41, 31], [-35, 35]])

finalize(globals())
