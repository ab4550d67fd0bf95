"""car_park (kinematic bicycle, parking between boxes) system config (reference: conf_car_park.py).

State (x, y, theta, v, delta, t); controls (acceleration, steering rate); CarPark.simulate
(environment.py:584-595) with the smooth-box obstacle reward over 10 body check points
(environment.py:604-641). The reference ships PER alpha = 0; BASELINE config C4 runs it with
alpha = 0.6 (set prioritized_replay_alpha before building the buffer)."""
import math
import numpy as np
from ._common import finalize

system_id = 'car_park'
EP_UPDATE = 200
UPDATE_LOOPS = np.arange(1000, 38000, 3000)
NUPDATES = 260000
NSTEPS = 100
BATCH_SIZE = 64
TD_DIV = 2
save_interval = 10000
plot_flag = 0
prioritized_replay_eps = 1e-2
fresh_factor = 0.95

XC1, YC1, A1, B1 = -10, 6.75, 17, 4.5
XC2, YC2, A2, B2 = 10, 6.75, 17, 4.5
XC3, YC3, A3, B3 = 0, -2, 40, 4
obs_param = np.array([XC1, YC1, XC2, YC2, XC3, YC3, A1, B1, A2, B2, A3, B3])
L = 4.35
W = 2
L_delta = 2.63
tau_delta = 1
check_points_BF = np.array([[-L / 2, W / 2], [-L / 2 + L / 3, W / 2], [-L / 2 + 2 / 3 * L, W / 2], [L / 2, W / 2],
                            [L / 2, 0], [L / 2, -W / 2], [-L / 2 + 2 / 3 * L, -W / 2], [-L / 2 + L / 3, -W / 2],
                            [-L / 2, -W / 2], [-L / 2, 0]])
w_d, w_u, w_peak, w_ob, w_v = 1e2, 1e1, 1e6, 5e4, 1e2
delta_bound = 2 * np.pi / 6
w_delta_bound = 0
cost_weights_running = np.array([w_d, w_peak, 0., w_ob, w_ob, w_ob, w_u, w_delta_bound])
cost_weights_terminal = np.array([w_d, w_peak, w_v, w_ob, w_ob, w_ob, 0, w_delta_bound])
k_db = 50
alpha, alpha2 = 50, 1
x_des, y_des = 0, 6.75
TARGET_STATE = np.array([x_des, y_des])

dt = 0.05
nb_state = 5 + 1
nq = None
nv = None
nx = 5
na = 2
tau_coulomb_max = 0 * np.ones(2)
x_min = np.array([-np.inf, -np.inf, -np.inf, -np.inf, -np.inf, 0])
x_init_min = np.array([-10, 1.5, -math.pi / 6, 0, 0, 0])
x_max = np.array([np.inf] * 6)
x_init_max = np.array([10, 3, math.pi / 6, 0, 0, (NSTEPS - 1) * dt])
state_norm_arr = np.array([10, 3, math.pi, 10, math.pi / 6, int(NSTEPS * dt)])
init_states_sim = [np.array([x - L_delta, 2.0, 0.0, 0.0, 0.0, 0.0]) for x in (-9.0, -5.0, -2.5, 0.0, 2.5, 5.0, 9.0)]
acc_lower_bound, acc_upper_bound = -3, 3
delta_dot_lower_bound, delta_dot_upper_bound = -1, 1
u_min = np.array([acc_lower_bound, delta_dot_lower_bound])
u_max = np.array([acc_upper_bound, delta_dot_upper_bound])
fig_ax_lim = np.array([[-11, 11], [-2.5, 10]])

finalize(globals())
