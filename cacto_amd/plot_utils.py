"""Policy evaluation with the reference surface of PLOT (plot_utils.py:245-279), on the GPU.

`PLOT.rollout` rolls the actor out from every state of `init_states_sim` for the full NSTEPS
(no NSTEPS_SH shortening) with the running weights, all episodes in one `cacto_rollout` launch,
and returns the reference's `returns` dict {(x0, y0): episodic reward}. The episodic reward is
Python's left-to-right float sum of the per-step rewards, as `rollout_episodic_reward += rwrd_sim`
accumulates it. The end-effector trajectories keep the reference's quirk
`rollout_p_ee[i+1, -1] = rollout_states[i+1, 2]` (plot_utils.py:265) and are left in
`self.p_ee_all_sim` for a caller that plots them; figure drawing itself is out of scope.
"""
import numpy as np


class PLOT:
    def __init__(self, N_try, env, NN, conf, learner=None):
        self.N_try = N_try
        self.env = env
        self.NN = NN
        self.conf = conf
        self.learner = learner            # the RL_AC that owns the device rollout (cacto_amd.rl)
        self.p_ee_all_sim = []
        self.states_all_sim = []

    def rollout(self, update_step_cntr, actor_model, init_states_sim, diff_loc=0):
        """plot_utils.py:245-279."""
        if self.learner is None:
            raise RuntimeError("PLOT.rollout needs the RL_AC learner that runs cacto_rollout")
        S0 = np.asarray([np.asarray(s, dtype=np.float64) for s in init_states_sim])
        n = len(S0)
        T = int(self.conf.NSTEPS)
        out = self.learner.rollout_batch(S0, [T] * n, T, ep=1, weights=self.conf.cost_weights_running,
                                         want=("S", "R", "EE"), actor=actor_model)
        S = out["S"].cpu().numpy()
        R = out["R"].cpu().numpy()
        EE = out["EE"].cpu().numpy()
        returns = {}
        self.p_ee_all_sim, self.states_all_sim = [], []
        for k in range(n):
            p_ee = EE[k].copy()
            p_ee[1:, -1] = S[k, 1:, 2]                    # plot_utils.py:265
            ret = 0
            for r in R[k]:                                # plot_utils.py:267, Python float accumulation
                ret += float(r)
            if k == 0:
                print("N try = {}: Simulation Return @ N updates = {} ==> {}".format(self.N_try, update_step_cntr,
                                                                                    ret))
            self.p_ee_all_sim.append(p_ee)
            self.states_all_sim.append(S[k])
            returns[init_states_sim[k][0], init_states_sim[k][1]] = ret
        return returns
