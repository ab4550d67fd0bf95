"""car (kinematic unicycle with jerk input) system config (reference: conf_car.py).

State (x, y, theta, v, a, t); controls (omega, jerk); Car.simulate (environment.py:437-448) with the
three-ellipse planar reward (environment.py:457-480)."""
import math
import numpy as np
from ._common import finalize

system_id = 'car'
EP_UPDATE = 250
UPDATE_LOOPS = np.arange(1000, 38000, 3000)
NUPDATES = 260000
NSTEPS = 500
BATCH_SIZE = 64
TD_DIV = 4
save_interval = 10000
plot_flag = 1
prioritized_replay_eps = 1e-2
fresh_factor = 0.95

XC1, YC1, A1, B1 = -2.0, 0.0, 6, 10
XC2, YC2, A2, B2 = 3.0, 4.0, 12, 4
XC3, YC3, A3, B3 = 3.0, -4.0, 12, 4
obs_param = np.array([XC1, YC1, XC2, YC2, XC3, YC3, A1, B1, A2, B2, A3, B3])
w_d, w_u, w_peak, w_ob, w_v = 1e2, 1e1, 5e5, 5e6, 0
cost_weights_running = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, w_u])
cost_weights_terminal = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, 0])
alpha, alpha2 = 50, 5
x_des, y_des = -7.0, 0.0
TARGET_STATE = np.array([x_des, y_des])

dt = 0.05
nb_state = 5 + 1
nq = None
nv = None
nx = 5
na = 2
tau_coulomb_max = 0 * np.ones(2)
x_min = np.array([-np.inf, -np.inf, -np.inf, -np.inf, -np.inf, 0])
x_init_min = np.array([-15, -15, -math.pi, -10, -3, 0])
x_max = np.array([np.inf] * 6)
x_init_max = np.array([15, 15, math.pi, 10, 3, (NSTEPS - 1) * dt])
state_norm_arr = np.array([15, 15, math.pi, 10, 3, int(NSTEPS * dt)])
init_states_sim = [np.array([x, y, 0.0, 0.0, 0.0, 0.0]) for x, y in (
    (2.0, 0.0), (10.0, 0.0), (10.0, -10.0), (10.0, 10.0), (-10.0, 10.0), (-10.0, -10.0), (12.0, 2.0),
    (12.0, -2.0), (15.0, 0.0))]
omega_lower_bound, omega_upper_bound = -2, 2
jerk_lower_bound, jerk_upper_bound = -1, 1
u_min = np.array([omega_lower_bound, jerk_lower_bound])
u_max = np.array([omega_upper_bound, jerk_upper_bound])
fig_ax_lim = np.array([[-16, 16], [-16, 16]])

finalize(globals())
