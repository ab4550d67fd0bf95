"""Minimal URDF -> joint-table parser (replaces `RobotWrapper.BuildFromURDF`, conf_*.py:157-165).

Supports what the reference's three URDFs use: `revolute`/`continuous`/`prismatic`/`fixed` joints,
`<origin xyz rpy>`, `<axis>`, and `<inertial>` (mass, origin, inertia tensor). As in Pinocchio:
  * every fixed joint becomes a frame; its child's inertia is merged into the nearest movable
    ancestor body and its placement is composed into the children's joint placements;
  * movable joints are numbered depth-first from the root link (Pinocchio's joint order);
  * frame 'EE' (or any requested frame) is located by its parent movable joint + fixed placement.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Tuple

import numpy as np

from .robots import PRISMATIC, REVOLUTE, Joint, RobotModel, rpy_to_matrix


def _origin(el) -> Tuple[np.ndarray, np.ndarray]:
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.eye(3), np.zeros(3)
    xyz = np.array([float(v) for v in o.get("xyz", "0 0 0").split()])
    rpy = [float(v) for v in o.get("rpy", "0 0 0").split()]
    return rpy_to_matrix(*rpy), xyz


def _inertial(link) -> Tuple[float, np.ndarray, np.ndarray]:
    """(mass, com, inertia about COM expressed in the link frame)."""
    iel = link.find("inertial")
    if iel is None:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    R, c = _origin(iel)
    m = float(iel.find("mass").get("value"))
    t = iel.find("inertia")
    g = lambda k: float(t.get(k, "0"))
    Ic = np.array([[g("ixx"), g("ixy"), g("ixz")],
                   [g("ixy"), g("iyy"), g("iyz")],
                   [g("ixz"), g("iyz"), g("izz")]])
    return m, c, R @ Ic @ R.T


def _merge(m1, c1, I1, m2, c2, I2):
    """Sum of two rigid bodies' inertias (parallel-axis theorem), all in one frame."""
    m = m1 + m2
    if m == 0.0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    c = (m1 * c1 + m2 * c2) / m
    def shift(mi, ci):
        d = ci - c
        return mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return m, c, I1 + shift(m1, c1) + I2 + shift(m2, c2)


def parse_urdf(source: str, ee_frame: str = "EE", name: Optional[str] = None) -> RobotModel:
    """Parse a URDF file path or XML string into a RobotModel."""
    if source.lstrip().startswith("<"):
        root = ET.fromstring(source)
    else:
        root = ET.parse(source).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    children: Dict[str, List] = {}
    child_links = set()
    for j in root.findall("joint"):
        children.setdefault(j.find("parent").get("link"), []).append(j)
        child_links.add(j.find("child").get("link"))
    roots = [n for n in links if n not in child_links]
    if len(roots) != 1:
        raise ValueError("URDF must have exactly one root link, found %s" % roots)

    joints: List[Joint] = []
    ee = None

    # Walk depth-first. State: (link name, parent movable joint index, placement of this link's
    # frame in the parent movable joint's frame).
    def visit(link_name: str, parent_idx: int, R: np.ndarray, p: np.ndarray):
        nonlocal ee
        m, c, I = _inertial(links[link_name])
        if m != 0.0:
            c_in = R @ c + p
            I_in = R @ I @ R.T
            if parent_idx >= 0:
                jb = joints[parent_idx]
                jb.mass, jb.com, jb.inertia = _merge(jb.mass, jb.com, jb.inertia, m, c_in, I_in)
            # inertia attached to the universe does not enter the dynamics of a fixed-base robot
        if link_name == ee_frame:
            ee = (parent_idx, R.copy(), p.copy())
        for jel in children.get(link_name, []):
            Rj, pj = _origin(jel)
            Rc, pc = R @ Rj, R @ pj + p
            kind = jel.get("type")
            child = jel.find("child").get("link")
            if kind == "fixed":
                visit(child, parent_idx, Rc, pc)
                continue
            if kind in ("revolute", "continuous"):
                jt = REVOLUTE
            elif kind == "prismatic":
                jt = PRISMATIC
            else:
                raise ValueError("unsupported joint type %r" % kind)
            ax_el = jel.find("axis")
            axis = np.array([float(v) for v in ax_el.get("xyz").split()]) if ax_el is not None \
                else np.array([1.0, 0.0, 0.0])
            axis = axis / np.linalg.norm(axis)
            joints.append(Joint(jel.get("name"), parent_idx, jt, axis, Rc, pc))
            visit(child, len(joints) - 1, np.eye(3), np.zeros(3))

    visit(roots[0], -1, np.eye(3), np.zeros(3))
    if ee is None:
        raise ValueError("frame %r not found in URDF" % ee_frame)
    return RobotModel(name or root.get("name", "robot"), joints, ee[0], ee[1], ee[2])
