"""Oracle: rigid-body dynamics of a serial chain (test infrastructure only — see oracle/__init__).

Restates what the reference gets from Pinocchio 2.9.2 (`pin3x-jnrh2023==2.9.2`, requirements.txt:218;
not vendored, not installed here):
  * `pin.computeAllTerms` -> data.M (CRBA) and data.nle (RNEA with zero acceleration, gravity
    included), used by `RobotSimulator.step` (robot_utils.py:353-356, :399-405);
  * `pin.computeABADerivatives(...).Minv` (environment.py:100-103) -> M(q)^-1;
  * `robot.framePlacement(q, 'EE').translation` (environment.py:146-156).
Published algorithms: Featherstone, "Rigid Body Dynamics Algorithms" (2008), RNEA Table 5.1 and
CRBA Table 6.2, with Pinocchio's spatial-vector ordering (linear, angular). This version uses plain
6x6 spatial matrices (the GPU kernel uses a compact form), so it is an independent restatement.

Input: the float64 joint table of `cacto_joint_t` (one row per joint: parent, type, axis[3],
R[9], p[3], mass, com[3], I[6]) plus the EE frame (parent, R, p) and gravity.
"""
import numpy as np

REVOLUTE, PRISMATIC = 0, 1


def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def _rot(axis, q):
    """Rotation by angle q about unit axis (Rodrigues)."""
    K = _skew(axis)
    return np.eye(3) + np.sin(q) * K + (1.0 - np.cos(q)) * (K @ K)


def _Xmotion(R, p):
    """6x6 motion transform for SE3 (R, p) mapping child-frame motions into the parent frame:
    act(v) = (R v_lin + p x (R v_ang), R v_ang)."""
    X = np.zeros((6, 6), dtype=np.result_type(R, p))
    X[:3, :3] = R
    X[:3, 3:] = _skew(p) @ R
    X[3:, 3:] = R
    return X


def _Xforce(R, p):
    """6x6 force transform (child -> parent): act(f) = (R f_lin, R f_ang + p x (R f_lin))."""
    X = np.zeros((6, 6), dtype=np.result_type(R, p))
    X[:3, :3] = R
    X[3:, :3] = _skew(p) @ R
    X[3:, 3:] = R
    return X


def _inertia6(m, c, Ic):
    """6x6 spatial inertia at the body origin, (lin, ang) ordering."""
    C = _skew(c)
    I = np.zeros((6, 6))
    I[:3, :3] = m * np.eye(3)
    I[:3, 3:] = -m * C
    I[3:, :3] = m * C
    I[3:, 3:] = Ic - m * C @ C
    return I


def _crm(v):
    """Motion cross-product matrix v x (.)."""
    X = np.zeros((6, 6), dtype=v.dtype)
    X[:3, :3] = _skew(v[3:])
    X[:3, 3:] = _skew(v[:3])
    X[3:, 3:] = _skew(v[3:])
    return X


def _crf(v):
    return -_crm(v).T


class Chain:
    def __init__(self, table, ee_parent, ee_R, ee_p, gravity=(0.0, 0.0, -9.81)):
        t = np.asarray(table, dtype=np.float64)
        self.n = t.shape[0]
        self.parent = [int(r[0]) for r in t]
        self.kind = [int(r[1]) for r in t]
        self.axis = [r[2:5].copy() for r in t]
        self.R0 = [r[5:14].reshape(3, 3).copy() for r in t]
        self.p0 = [r[14:17].copy() for r in t]
        self.I6 = []
        for r in t:
            Ic = np.array([[r[21], r[22], r[23]], [r[22], r[24], r[25]], [r[23], r[25], r[26]]])
            self.I6.append(_inertia6(r[17], r[18:21], Ic))
        self.ee_parent = int(ee_parent)
        self.ee_R = np.asarray(ee_R, dtype=np.float64)
        self.ee_p = np.asarray(ee_p, dtype=np.float64)
        self.gravity = np.asarray(gravity, dtype=np.float64)

    @classmethod
    def from_model(cls, model):
        return cls(model.table(), model.ee_parent, model.ee_R, model.ee_p, model.gravity)

    def _S(self, i):
        S = np.zeros(6)
        if self.kind[i] == REVOLUTE:
            S[3:] = self.axis[i]
        else:
            S[:3] = self.axis[i]
        return S

    def _placement(self, i, qi):
        """(R, p) of joint i's frame in its parent's frame: jointPlacement * J(q)."""
        if self.kind[i] == REVOLUTE:
            return self.R0[i] @ _rot(self.axis[i], qi), self.p0[i].copy()
        return self.R0[i].copy(), self.p0[i] + self.R0[i] @ (self.axis[i] * qi)

    def mass_matrix(self, q):
        """CRBA (Featherstone Table 6.2)."""
        n = self.n
        Xm, Xf = [], []
        for i in range(n):
            R, p = self._placement(i, q[i])
            Xm.append(_Xmotion(R, p))
            Xf.append(_Xforce(R, p))
        Ic = [I.astype(Xm[0].dtype) for I in self.I6]
        for i in range(n - 1, -1, -1):
            if self.parent[i] >= 0:
                # composite inertia expressed in parent: Xf Ic Xm^-1
                Ic[self.parent[i]] += Xf[i] @ Ic[i] @ np.linalg.inv(Xm[i])
        M = np.zeros((n, n), dtype=Xm[0].dtype)
        for i in range(n):
            F = Ic[i] @ self._S(i)
            M[i, i] = self._S(i) @ F
            j = i
            while self.parent[j] >= 0:
                F = Xf[j] @ F
                j = self.parent[j]
                M[i, j] = M[j, i] = self._S(j) @ F
        return M

    def nle(self, q, v):
        """RNEA with qdd = 0: h = C(q, v) v + g(q) (Featherstone Table 5.1, a_0 = -gravity)."""
        return self.rnea(q, v, np.zeros(self.n))

    def rnea(self, q, v, qdd):
        """tau = M(q) qdd + h(q, v) (Featherstone Table 5.1). Works on complex inputs too (the
        complex-step derivatives of oracle/ddp.py)."""
        n = self.n
        vel, acc, f, Xm, Xf = [], [], [], [], []
        for i in range(n):
            R, p = self._placement(i, q[i])
            Xm.append(_Xmotion(R, p))
            Xf.append(_Xforce(R, p))
            Xinv = np.linalg.inv(Xm[i])
            S = self._S(i)
            if self.parent[i] < 0:
                vp = np.zeros(6)
                ap = np.concatenate([-self.gravity, np.zeros(3)])
            else:
                vp, ap = vel[self.parent[i]], acc[self.parent[i]]
            vi = Xinv @ vp + S * v[i]
            ai = Xinv @ ap + _crm(vi) @ (S * v[i]) + S * qdd[i]
            vel.append(vi)
            acc.append(ai)
            f.append(self.I6[i] @ ai + _crf(vi) @ (self.I6[i] @ vi))
        tau = np.zeros(n, dtype=np.result_type(*f))
        for i in range(n - 1, -1, -1):
            tau[i] = self._S(i) @ f[i]
            if self.parent[i] >= 0:
                f[self.parent[i]] = f[self.parent[i]] + Xf[i] @ f[i]
        return tau

    def frame_position(self, q):
        """Translation of the EE frame in the world (forward kinematics)."""
        n = self.n
        oR = [None] * n
        op = [None] * n
        for i in range(n):
            R, p = self._placement(i, q[i])
            if self.parent[i] < 0:
                oR[i], op[i] = R, p
            else:
                pr = self.parent[i]
                oR[i], op[i] = oR[pr] @ R, oR[pr] @ p + op[pr]
        j = self.ee_parent
        return oR[j] @ self.ee_p + op[j]
