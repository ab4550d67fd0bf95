"""Rigid-body chain models for the robot systems (joint tables fed to the HIP dynamics kernels).

The reference builds a Pinocchio model from a URDF at conf-import time
(`conf_double_integrator.py:157-165`, `conf_manipulator.py:157-165`, `conf_ur5.py:168-177`) and the
RL environment only ever asks it for M(q), nle(q, v) (`robot_utils.py:353-356`), Minv
(`environment.py:100-103`) and the placement of the frame 'EE' (`environment.py:146-156`).
Those quantities depend only on a serial chain of 1-DoF joints, so a model here is:

  * one `Joint` per actuated joint, in Pinocchio's depth-first order: parent joint index (-1 =
    universe), joint type, unit axis in the joint frame, the fixed placement (R, p) of the joint
    frame in the parent joint's frame (every fixed URDF joint on the way composed in), and the body
    inertia (mass, centre of mass, rotational inertia about the COM, in the joint frame) with every
    fixed child link's inertia merged in, as Pinocchio does for fixed joints;
  * the 'EE' frame: parent joint and fixed placement;
  * gravity (Pinocchio's default model.gravity = [0, 0, -9.81]).

`builtin_model(name)` returns the tables for the systems the reference ships without needing the
URDF files at run time; `cacto_amd.urdf.parse_urdf` builds the same tables from a URDF and the CPU
test suite checks the two agree on the reference's own files.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List

import numpy as np

REVOLUTE = 0
PRISMATIC = 1


@dataclass
class Joint:
    name: str
    parent: int
    kind: int
    axis: np.ndarray
    R: np.ndarray          # 3x3 placement rotation in the parent joint frame
    p: np.ndarray          # placement translation in the parent joint frame
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about COM


@dataclass
class RobotModel:
    name: str
    joints: List[Joint]
    ee_parent: int
    ee_R: np.ndarray
    ee_p: np.ndarray
    gravity: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -9.81]))

    @property
    def nq(self) -> int:
        return len(self.joints)

    @property
    def nv(self) -> int:
        return len(self.joints)

    @property
    def na(self) -> int:
        # RobotWrapper.na = nv for fixed-base robots (robot_utils.py:241 builds S = [0 | I_na])
        return len(self.joints)

    def table(self) -> np.ndarray:
        """Pack into the float64 joint table layout of `cacto_joint_t` (include/cacto_hip.h)."""
        rows = []
        for j in self.joints:
            I = j.inertia
            rows.append(np.concatenate([
                [float(j.parent), float(j.kind)], j.axis, j.R.reshape(-1), j.p, [j.mass], j.com,
                [I[0, 0], I[0, 1], I[0, 2], I[1, 1], I[1, 2], I[2, 2]]]))
        return np.asarray(rows, dtype=np.float64)


def rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """URDF rpy convention (fixed axes X, Y, Z): R = Rz(y) Ry(p) Rx(r) (same as pinocchio.rpy)."""
    cr, sr = math.cos(r), math.sin(r)
    cp, sp = math.cos(p), math.sin(p)
    cy, sy = math.cos(y), math.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _double_integrator() -> RobotModel:
    # urdf/double_integrator.urdf: world -slider_x(prismatic X)-> Sx -slider_y(prismatic Y)-> Sy
    # -fixed-> EE carrying the only inertia (m = 1, izz = 1, COM at the EE origin).
    eye = np.eye(3)
    j0 = Joint("slider_x", -1, PRISMATIC, np.array([1.0, 0, 0]), eye.copy(), np.zeros(3))
    j1 = Joint("slider_y", 0, PRISMATIC, np.array([0, 1.0, 0]), eye.copy(), np.zeros(3),
               mass=1.0, com=np.zeros(3), inertia=np.diag([0.0, 0.0, 1.0]))
    return RobotModel("double_integrator", [j0, j1], 1, eye.copy(), np.zeros(3))


def _planar_manipulator_3dof() -> RobotModel:
    # urdf/planar_manipulator_3dof.urdf: base fixed at x = -7; three revolute-Z links of length 10,
    # m = 0.5, COM at x = 5, ixx = izz = 16.666..., iyy = 0; EE fixed 10 along x of link_2.
    eye = np.eye(3)
    I = np.diag([16.666666666666668, 0.0, 16.666666666666668])
    joints = []
    for k in range(3):
        p = np.array([-7.0, 0.0, 0.0]) if k == 0 else np.array([10.0, 0.0, 0.0])
        joints.append(Joint("joint_%d" % k, k - 1, REVOLUTE, np.array([0, 0, 1.0]), eye.copy(), p,
                            mass=0.5, com=np.array([5.0, 0.0, 0.0]), inertia=I.copy()))
    return RobotModel("planar_manipulator_3dof", joints, 2, eye.copy(), np.array([10.0, 0.0, 0.0]))


def _ur5() -> RobotModel:
    # urdf/ur5_robot.urdf (example-robot-data UR5): six revolute joints in a serial chain, every link
    # inertia diagonal about its COM; EE fixed to wrist_3_link at xyz (0, 0.0823, 0), rpy (0, 0, 1.57079632679).
    # Literal URDF numbers (the pitch 1.57079632679 is not exactly pi/2; kept as written).
    hp = 1.57079632679
    spec = [  # name, axis, rpy, xyz, mass, com, (ixx, iyy, izz)
        ("shoulder_pan_joint", (0, 0, 1), (0, 0, 0), (0.0, 0.0, 0.089159), 3.7, (0, 0, 0),
         (0.010267495893, 0.010267495893, 0.00666)),
        ("shoulder_lift_joint", (0, 1, 0), (0, hp, 0), (0.0, 0.13585, 0.0), 8.393, (0, 0, 0.28),
         (0.22689067591, 0.22689067591, 0.0151074)),
        ("elbow_joint", (0, 1, 0), (0, 0, 0), (0.0, -0.1197, 0.425), 2.275, (0, 0, 0.25),
         (0.049443313556, 0.049443313556, 0.004095)),
        ("wrist_1_joint", (0, 1, 0), (0, hp, 0), (0.0, 0.0, 0.39225), 1.219, (0, 0, 0),
         (0.111172755531, 0.111172755531, 0.21942)),
        ("wrist_2_joint", (0, 0, 1), (0, 0, 0), (0.0, 0.093, 0.0), 1.219, (0, 0, 0),
         (0.111172755531, 0.111172755531, 0.21942)),
        ("wrist_3_joint", (0, 1, 0), (0, 0, 0), (0.0, 0.0, 0.09465), 0.1879, (0, 0, 0),
         (0.0171364731454, 0.0171364731454, 0.033822)),
    ]
    joints = []
    for k, (name, axis, rpy, xyz, m, com, I) in enumerate(spec):
        joints.append(Joint(name, k - 1, REVOLUTE, np.array(axis, dtype=np.float64), rpy_to_matrix(*rpy),
                            np.array(xyz, dtype=np.float64), mass=m, com=np.array(com, dtype=np.float64),
                            inertia=np.diag(np.array(I, dtype=np.float64))))
    return RobotModel("ur5", joints, 5, rpy_to_matrix(0.0, 0.0, hp), np.array([0.0, 0.0823, 0.0]))


_BUILTIN = {
    "double_integrator": _double_integrator,
    "planar_manipulator_3dof": _planar_manipulator_3dof,
    "ur5": _ur5,
}


def builtin_model(name: str) -> RobotModel:
    try:
        return _BUILTIN[name]()
    except KeyError:
        raise KeyError("no built-in robot model %r (have: %s); build one with "
                       "cacto_amd.urdf.parse_urdf" % (name, ", ".join(sorted(_BUILTIN))))
