"""Oracle: actor/critic MLPs, Sobolev critic gradient, actor gradient, Keras Adam, soft update
(test infrastructure only — see oracle/__init__).

Parameter lists follow Keras `trainable_variables` order: [kernel0 [in,out], bias0, kernel1, ...].

Restated:
  * normalize_tensor                      utils.py:17-24
  * actor  Dense-LeakyReLU(0.3)x2-Dense   NeuralNetwork.py:51-63 (regularisers never enter a loss)
  * critic 4x sin(xW+b) (tf_siren w0=1) + Dense(1)                       NeuralNetwork.py:95-108
    and the sine-elu critic (sine, elu, sine, elu hidden layers of the same widths)  :80-93
  * custom_logarithm                      NeuralNetwork.py:140-148
  * compute_critic_grad (Sobolev)         NeuralNetwork.py:150-178
  * compute_actor_grad                    NeuralNetwork.py:180-233
  * Keras-2.11 Adam update_step           RL.py:79-88, :105, :109 (keras optimizer_experimental)
  * update_target                         RL.py:113-118
All arithmetic here is float64 (the GPU computes float32; tests compare within stated tolerances).
"""
import numpy as np

LEAKY_ALPHA = 0.3      # keras.layers.LeakyReLU() default alpha
CLOG_EPS = 1e-7        # NeuralNetwork.py:142-143


def normalize(S, norm):
    """utils.py:17-24: s_i / norm_i for i < ns-1; time column t / norm_T * 2 - 1."""
    S = np.asarray(S, dtype=np.float64)
    out = S / norm
    out[:, -1] = S[:, -1] / norm[-1] * 2 - 1
    return out


def norm_grad_scale(norm):
    """d normalize(s)_i / d s_i."""
    g = 1.0 / np.asarray(norm, dtype=np.float64)
    g[-1] = 2.0 / norm[-1]
    return g


def lrelu(z):
    return np.where(z > 0, z, LEAKY_ALPHA * z)


def lrelu_grad(z):
    return np.where(z > 0, 1.0, LEAKY_ALPHA)


def actor_forward(params, S, norm, keep=False):
    W1, b1, W2, b2, W3, b3 = [np.asarray(p, dtype=np.float64) for p in params]
    x0 = normalize(S, norm)
    z1 = x0 @ W1 + b1
    h1 = lrelu(z1)
    z2 = h1 @ W2 + b2
    h2 = lrelu(z2)
    a = h2 @ W3 + b3
    if keep:
        return a, (x0, z1, h1, z2, h2)
    return a


def actor_forward32(params, S, norm):
    """The actor as TF runs it (NeuralNetwork.py:51-63, NN.eval :130-138): float32 tensors and
    float32 ops throughout, so IEEE float32 overflow / inf / NaN propagate as in the reference
    (the float64 `actor_forward` above cannot overflow where the reference does). Normalisation in
    float32 (RealDiv, then *2 - 1 for the time column, utils.py:17-24)."""
    f32 = np.float32
    W1, b1, W2, b2, W3, b3 = [np.asarray(p, dtype=f32) for p in params]
    x = np.asarray(S, dtype=f32).copy()
    nm = np.asarray(norm, dtype=f32)
    with np.errstate(over="ignore", invalid="ignore"):
        x[:, :-1] = x[:, :-1] / nm[:-1]
        x[:, -1] = x[:, -1] / nm[-1] * f32(2) - f32(1)
        z1 = x @ W1 + b1
        h1 = np.where(z1 > 0, z1, z1 * f32(LEAKY_ALPHA))
        z2 = h1 @ W2 + b2
        h2 = np.where(z2 > 0, z2, z2 * f32(LEAKY_ALPHA))
        return h2 @ W3 + b3


SINE = ("sine",) * 4            # critic_type 'sine' (every shipped config)
SINE_ELU = ("sine", "elu", "sine", "elu")   # critic_type 'sine-elu' (NeuralNetwork.py:80-93)


def act(z, kind):
    """Hidden activation: tf_siren sin(z) (w0 = 1) or Keras 'elu' (z if z > 0 else exp(z) - 1)."""
    return np.sin(z) if kind == "sine" else np.where(z > 0, z, np.expm1(np.minimum(z, 0.0)))


def act_d1(z, kind):
    return np.cos(z) if kind == "sine" else np.where(z > 0, 1.0, np.exp(np.minimum(z, 0.0)))


def act_d2(z, kind):
    return -np.sin(z) if kind == "sine" else np.where(z > 0, 0.0, np.exp(np.minimum(z, 0.0)))


def critic_forward(params, S, norm, keep=False, acts=SINE):
    P = [np.asarray(p, dtype=np.float64) for p in params]
    h = normalize(S, norm)
    hs, zs = [h], []
    for l in range(4):
        z = h @ P[2 * l] + P[2 * l + 1]
        h = act(z, acts[l])
        zs.append(z)
        hs.append(h)
    V = h @ P[8] + P[9]
    if keep:
        return V, (hs, zs)
    return V


def critic_input_grad(params, S, norm, keep=None, acts=SINE):
    """dV/ds (raw state) through the MLP (activation derivatives) and the normalisation."""
    P = [np.asarray(p, dtype=np.float64) for p in params]
    if keep is None:
        _, keep = critic_forward(params, S, norm, keep=True, acts=acts)
    hs, zs = keep
    g = np.broadcast_to(P[8][:, 0], (S.shape[0], P[8].shape[0]))
    ds = []
    for l in range(3, -1, -1):
        d = g * act_d1(zs[l], acts[l])
        ds.append(d)
        g = d @ P[2 * l].T
    ds = ds[::-1]          # ds[l] = dV/dz_{l+1}
    return g * norm_grad_scale(norm), ds


def clog(x):
    return np.where(x > 0, np.log(np.maximum(x, CLOG_EPS) + 1), -np.log(np.maximum(-x, CLOG_EPS) + 1))


def clog_grad(x):
    ax = np.abs(x)
    return np.where(ax >= CLOG_EPS, 1.0 / (np.maximum(ax, CLOG_EPS) + 1.0), 0.0)


def compute_critic_grad(critic, target, S, S_next, R, dVdx, d, w, w_S, norm, MC=False, acts=SINE):
    """NeuralNetwork.py:150-178. Returns (grads, y, V, V_tgt(s), loss)."""
    S = np.asarray(S, dtype=np.float64)
    B = S.shape[0]
    R = np.asarray(R, dtype=np.float64).reshape(B, 1)
    d = np.asarray(d, dtype=np.float64).reshape(B, 1)
    w = np.asarray(w, dtype=np.float64).reshape(B, 1)
    if MC:
        y = R
    else:
        y = R + (1 - d) * critic_forward(target, S_next, norm, acts=acts)
    P = [np.asarray(p, dtype=np.float64) for p in critic]
    V, keep = critic_forward(critic, S, norm, keep=True, acts=acts)
    hs, zs = keep
    grads = [np.zeros_like(p) for p in P]
    zbar = [np.zeros_like(z) for z in zs]
    # value loss  w_S * (1/B) sum_b w_b (y - V)^2   (or its plain form when w_S == 0)
    wv = w_S if w_S != 0 else 1.0
    Vbar = wv * (2.0 / B) * w * (V - y)                       # [B,1]
    loss = wv * np.mean(w[:, 0] * (y - V)[:, 0] ** 2)
    grads[8] += hs[4].T @ Vbar
    grads[9] += Vbar.sum(axis=0)
    hbar = Vbar @ P[8].T
    if w_S != 0:
        dVds, ds = critic_input_grad(critic, S, norm, keep, acts=acts)
        ns = S.shape[1]
        yt, yp = clog(np.asarray(dVdx, dtype=np.float64)[:, :-1]), clog(dVds[:, :-1])
        loss += np.mean(w[:, 0] * np.mean((yp - yt) ** 2, axis=1))
        gyp = w * (2.0 / (B * (ns - 1))) * (yp - yt)           # dL/d clog(dVds)
        g0bar = np.zeros_like(dVds)
        g0bar[:, :-1] = gyp * clog_grad(dVds[:, :-1])
        gbar = g0bar * norm_grad_scale(norm)                   # adjoint of g_0 = dV/dx0
        # backward of the first backward pass. With G[4] = W5[:, 0], D[l] = G[l+1]*act'(z_l),
        # G[l] = D[l] W_l^T (G[0] = dV/dx0), walk l = 0..3 carrying gbar = adjoint of G[l].
        for l in range(4):
            W = P[2 * l]
            grads[2 * l] += gbar.T @ ds[l]                     # G[l] = D[l] W_l^T
            dbar = gbar @ W                                    # adjoint of D[l]
            g_up = _g_of_layer(P, zs, l, acts)                 # G[l+1]
            zbar[l] += dbar * g_up * act_d2(zs[l], acts[l])
            gbar = dbar * act_d1(zs[l], acts[l])               # adjoint of G[l+1]
        grads[8][:, 0] += gbar.sum(axis=0)                     # G[4] = W5[:, 0]
    # backward through the forward graph
    zbar[3] += hbar * act_d1(zs[3], acts[3])
    for l in range(3, -1, -1):
        grads[2 * l] += hs[l].T @ zbar[l]
        grads[2 * l + 1] += zbar[l].sum(axis=0)
        if l > 0:
            zbar[l - 1] += (zbar[l] @ P[2 * l].T) * act_d1(zs[l - 1], acts[l - 1])
    return grads, y, V, critic_forward(target, S, norm, acts=acts), loss


def _g_of_layer(P, zs, l, acts=SINE):
    """g_l = dV/dh_{l+1} (h_{l+1} = act(z_l)) for layer index l in 0..3."""
    B = zs[0].shape[0]
    g = np.broadcast_to(P[8][:, 0], (B, P[8].shape[0]))
    for k in range(3, l, -1):
        g = (g * act_d1(zs[k], acts[k])) @ P[2 * k].T
    return g


def critic_loss(critic, target, S, S_next, R, dVdx, d, w, w_S, norm, acts=SINE):
    """Scalar loss (for finite-difference checks)."""
    return compute_critic_grad(critic, target, S, S_next, R, dVdx, d, w, w_S, norm, acts=acts)[4]


def actor_dq_da(env, actor, critic, S, term, norm, acts=SINE):
    """dQ/da of NeuralNetwork.py:185-215 (float64; env.simulate_batch/derivative_batch cast to f32
    as the reference does)."""
    conf = env.conf
    S32 = np.asarray(S, dtype=np.float32)
    A = actor_forward(actor, S32, norm).astype(np.float32)
    S_next = env.simulate_batch(S32, A)
    Fu = env.derivative_batch(S32, A).astype(np.float64)
    dVds_next, _ = critic_input_grad(critic, S_next.astype(np.float64), norm, acts=acts)
    term = np.asarray(term, dtype=np.float64).reshape(-1, 1)
    W = term @ np.reshape(conf.cost_weights_terminal, (1, -1)) + \
        (1 - term) @ np.reshape(conf.cost_weights_running, (1, -1))
    dr_da = env.dr_da(W, A)
    dQ_da = np.einsum('bs,bsa->ba', dVds_next, Fu) + dr_da
    return dQ_da, A, S_next, Fu, dVds_next, dr_da


def compute_actor_grad(env, actor, critic, S, term, norm, batch_size=None, acts=SINE):
    """NeuralNetwork.py:180-233: grads of mean_b(-dQ/da_b . pi(s_b)) w.r.t. actor params."""
    S = np.asarray(S, dtype=np.float64)
    B = S.shape[0] if batch_size is None else batch_size
    dQ_da = actor_dq_da(env, actor, critic, S, term, norm, acts=acts)[0]
    P = [np.asarray(p, dtype=np.float64) for p in actor]
    a, (x0, z1, h1, z2, h2) = actor_forward(actor, S, norm, keep=True)
    abar = -dQ_da / B
    g = [None] * 6
    g[4] = h2.T @ abar
    g[5] = abar.sum(axis=0)
    z2bar = (abar @ P[4].T) * lrelu_grad(z2)
    g[2] = h1.T @ z2bar
    g[3] = z2bar.sum(axis=0)
    z1bar = (z2bar @ P[2].T) * lrelu_grad(z1)
    g[0] = x0.T @ z1bar
    g[1] = z1bar.sum(axis=0)
    return g


class KerasAdam:
    """Keras 2.11 (optimizer_experimental) Adam.update_step, float64 restatement:
    m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
    theta -= (m * lr*sqrt(1 - b2^t)/(1 - b1^t)) / (sqrt(v) + eps), t = iterations + 1.
    `lr` may be a float or a PiecewiseConstantDecay (boundaries, values) evaluated at
    `iterations` before the increment."""

    def __init__(self, lr, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr = lr
        self.b1, self.b2, self.eps = beta_1, beta_2, epsilon
        self.iterations = 0
        self.m = None
        self.v = None

    def current_lr(self):
        if isinstance(self.lr, tuple):
            bounds, values = self.lr
            for b, val in zip(bounds, values):
                if self.iterations <= b:
                    return val
            return values[-1]
        return self.lr

    def apply(self, params, grads):
        if self.m is None:
            self.m = [np.zeros_like(np.asarray(p, dtype=np.float64)) for p in params]
            self.v = [np.zeros_like(np.asarray(p, dtype=np.float64)) for p in params]
        t = self.iterations + 1
        lr = self.current_lr()
        alpha = lr * np.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            g = np.asarray(g, dtype=np.float64)
            self.m[i] = self.m[i] + (g - self.m[i]) * (1 - self.b1)
            self.v[i] = self.v[i] + (g * g - self.v[i]) * (1 - self.b2)
            out.append(np.asarray(p, dtype=np.float64) - (self.m[i] * alpha) / (np.sqrt(self.v[i]) + self.eps))
        self.iterations += 1
        return out


def soft_update(target, source, tau):
    """RL.py:113-118: a <- b*tau + a*(1 - tau)."""
    return [np.asarray(b, dtype=np.float64) * tau + np.asarray(a, dtype=np.float64) * (1 - tau)
            for a, b in zip(target, source)]
