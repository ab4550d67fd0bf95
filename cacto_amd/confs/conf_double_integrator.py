"""double_integrator system config (reference: conf_double_integrator.py).

State (x, y, ẋ, ẏ, t); Pinocchio model from urdf/double_integrator.urdf (two prismatic joints
carrying a unit mass, so M = I and nle = 0); `robot`/`simu` are this build's chain model and
HIP-backed simulator handle (conf_double_integrator.py:157-177)."""
import numpy as np
from ._common import finalize
from ..robots import builtin_model

system_id = 'double_integrator'
UPDATE_LOOPS = np.arange(1000, 18000, 3000)
NUPDATES = 50000
NSTEPS = 200
BATCH_SIZE = 128
TD_DIV = 4
save_interval = 5000
plot_flag = 1
prioritized_replay_eps = 1e-4
fresh_factor = 1

XC1, YC1, A1, B1 = -2.0, 0.0, 6, 10
XC2, YC2, A2, B2 = 3.0, 4.0, 12, 4
XC3, YC3, A3, B3 = 3.0, -4.0, 12, 4
obs_param = np.array([XC1, YC1, XC2, YC2, XC3, YC3, A1, B1, A2, B2, A3, B3])
w_d, w_u, w_peak, w_ob, w_v = 100, 10, 5e5, 5e6, 0
cost_weights_running = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, w_u])
cost_weights_terminal = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, 0])
alpha, alpha2 = 50, 5
x_des, y_des = -7.0, 0.0
TARGET_STATE = np.array([x_des, y_des])

URDF_FILENAME = "double_integrator.urdf"
robot = builtin_model("double_integrator")
nq = robot.nq
nv = robot.nv
nx = nq + nv
na = robot.na
dt = 0.05
tau_coulomb_max = 0 * np.ones(robot.na)
q_init, v_init = np.array([-5, 0]), np.zeros(robot.nv)
nb_state = robot.nq + robot.nv + 1
x_min = np.array([-np.inf, -np.inf, -np.inf, -np.inf, dt])
x_init_min = np.array([-15, -15, -6, -6, dt])
x_max = np.array([np.inf, np.inf, np.inf, np.inf, np.inf])
x_init_max = np.array([15, 15, 6, 6, (NSTEPS - 1) * dt])
state_norm_arr = np.array([15, 15, 6, 6, int(NSTEPS * dt)])
init_states_sim = [np.array([x, y, 0.0, 0.0, 0.0]) for x, y in
                   ((2.0, 0.0), (10.0, 0.0), (10.0, -10.0), (10.0, 10.0), (-10.0, 10.0),
                    (-10.0, -10.0), (12.0, 2.0), (12.0, -2.0), (15.0, 0.0))]
tau_lower_bound, tau_upper_bound = -2, 2
u_min = tau_lower_bound * np.ones(robot.na)
u_max = tau_upper_bound * np.ones(robot.na)
fig_ax_lim = np.array([[-15, 15], [-15, 15]])

finalize(globals())
