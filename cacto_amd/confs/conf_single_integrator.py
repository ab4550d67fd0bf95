"""single_integrator system config (reference: conf_single_integrator.py).

State (x, y, t); action (ẋ, ẏ); analytic dynamics x' = x + dt·u (environment.py:235-243)."""
import numpy as np
from ._common import finalize

system_id = 'single_integrator'
UPDATE_LOOPS = np.arange(1000, 25000, 3000)
NUPDATES = 100000
NSTEPS = 100
BATCH_SIZE = 128
TD_DIV = 4
save_interval = 5000
plot_flag = 1
prioritized_replay_eps = 1e-2
fresh_factor = 0.95

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

dt = 0.05
tau_coulomb_max = 0 * np.ones(2)
nb_state = 2 + 1
nq = None
nv = None
nx = 2
na = 2
x_min = np.array([-np.inf, -np.inf, 0])
x_init_min = np.array([-15, -15, 0])
x_max = np.array([np.inf, np.inf, np.inf])
x_init_max = np.array([15, 15, (NSTEPS - 1) * dt])
state_norm_arr = np.array([15, 15, int(NSTEPS * dt)])
init_states_sim = [np.array(v) for v in ([2.0, 0.0, 0.0], [10.0, 0.0, 0.0], [10.0, -10.0, 0.0],
                                         [10.0, 10.0, 0.0], [-10.0, 10.0, 0.0], [-10.0, -10.0, 0.0],
                                         [12.0, 2.0, 0.0], [12.0, -2.0, 0.0], [15.0, 0.0, 0.0])]
tau_lower_bound, tau_upper_bound = -6, 6
u_min = tau_lower_bound * np.ones(2)
u_max = tau_upper_bound * np.ones(2)
fig_ax_lim = np.array([[-16, 16], [-16, 16]])

finalize(globals())
