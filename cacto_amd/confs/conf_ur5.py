"""ur5 (6-DoF arm) system config (reference: conf_ur5.py).

State (q[6], qdot[6], t); Pinocchio model from urdf/ur5_robot.urdf (built in: robots.builtin_model
('ur5')), full 3-D with gravity; 3-D ellipsoid obstacles and a 3-D target (environment.py:780-805)."""
import math
import numpy as np
from ._common import finalize
from ..robots import builtin_model

system_id = 'ur5'
UPDATE_LOOPS = np.arange(1000, 50000, 3000)
NUPDATES = 380000
NSTEPS = 100
BATCH_SIZE = 64
TD_DIV = 4
save_interval = 5000
plot_flag = 1
prioritized_replay_eps = 1e-2
fresh_factor = 0.95

XC1, YC1, ZC1 = 0.0, 0.25, 0.2
A1, B1, C1 = 0.5, 0.2, 0.34
XC2, YC2, ZC2 = 0.2, 0.425, 0.2
A2, B2, C2 = 0.4, 0.14, 0.34
XC3, YC3, ZC3 = -0.2, 0.425, 0.2
A3, B3, C3 = 0.4, 0.14, 0.34
ell1_center, ell2_center, ell3_center = [XC1, YC1, ZC1], [XC2, YC2, ZC2], [XC3, YC3, ZC3]
obs_param = np.array([XC1, YC1, ZC1, XC2, YC2, ZC2, XC3, YC3, ZC3, A1, B1, C1, A2, B2, C2, A3, B3, C3])
w_d, w_u, w_peak, w_ob, w_v = 100, 1, 5e5, 5e6, 0
cost_weights_running = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, w_u])
cost_weights_terminal = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, 0])
alpha, alpha2 = 50, 5
x_des, y_des, z_des = 0.0, 0.425, 0.2
TARGET_STATE = np.array([x_des, y_des, z_des])

URDF_FILENAME = "ur5_robot.urdf"
robot = builtin_model("ur5")
nq = robot.nq
nv = robot.nv
nx = nq + nv
na = robot.na
tau_coulomb_max = 0 * np.ones(robot.na)
q_init, v_init = np.array([0., -math.pi / 2, 0., 0., 0., 0.]), np.zeros(robot.nv)
dt = 0.01
nb_state = robot.nq + robot.nv + 1
_pi, _p4 = math.pi, math.pi / 4
x_min = np.array([-np.inf] * 12 + [0])
x_init_min = np.array([-_pi] * 6 + [-_p4] * 6 + [0])
x_max = np.array([np.inf] * 13)
x_init_max = np.array([_pi] * 6 + [_p4] * 6 + [(NSTEPS - 1) * dt])
state_norm_arr = np.array([10] * 12 + [int(NSTEPS * dt)])
init_states_sim = [np.array(list(q) + [0.0] * 10) for q in (
    (_pi / 4, -_pi / 8, -_pi / 8), (-_pi / 4, _pi / 8, _pi / 8), (_pi / 2, 0.0, 0.0), (-_pi / 2, 0.0, 0.0),
    (3 * _pi / 4, 0.0, 0.0), (-3 * _pi / 4, 0.0, 0.0), (_pi / 4, 0.0, 0.0), (-_pi / 4, 0.0, 0.0), (_pi, 0.0, 0.0))]
u_min = np.array([-150, -150, -150, -28, -28, -28])
u_max = np.array([150, 150, 150, 28, 28, 28])
fig_ax_lim = np.array([[-3, 3], [-3, 3]])

finalize(globals())
