# isolate cacto_env_jacobians for the UR5 chain: full wave first, then a partial wave
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cacto_amd.confs import load_conf
from cacto_amd.environment import make_env
conf = load_conf(sys.argv[1] if len(sys.argv) > 1 else "ur5")
env = make_env(conf)
rng = np.random.default_rng(0)
for B in (64, 40):
    S = rng.uniform(-1, 1, size=(B, conf.nb_state))
    A = rng.uniform(-1, 1, size=(B, conf.nb_action))
    print("launch B=%d" % B, flush=True)
    Fx, Fu = env.augmented_derivative_batch(S, A)
    torch.cuda.synchronize()
    print("ok B=%d" % B, float(Fx.abs().max()), float(Fu.abs().max()), flush=True)
