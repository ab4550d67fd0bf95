"""CPU-side checks of the drop-in boundary: the C-ABI library builds/loads and exports every
symbol include/cacto_hip.h declares; ctypes struct layouts match the header; host logic."""
import ctypes
import os
import re

import numpy as np
import pytest

from cacto_amd import _lib as L
from cacto_amd.confs import load_conf
from cacto_amd.robots import builtin_model
from cacto_amd.urdf import parse_urdf
from conftest import REFERENCE


def test_library_exports_every_header_symbol():
    lib = L.lib()
    names = L.header_exports()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib.dll, n)]
    assert not missing, missing
    assert lib.dll.cacto_abi_version() == 1


def test_struct_sizes_match_header():
    # sizes computed from the header's declarations (all int32 then doubles)
    assert ctypes.sizeof(L.SysParams) == 12 * 4 + 8 * (1 + 16 + 8 + 1 + 2 + 2 + 18 + 3 + 8 + 8 + 3 + 20 + 9 + 3 + 3)
    assert ctypes.sizeof(L.Nets) == 8 * 8
    assert ctypes.sizeof(L.UpdateCfg) == 8 * (5 + 5 + 5 + 4) + 4 * 4


def test_errors_are_reported_not_raised_in_c():
    lib = L.lib()
    p = L.SysParams()
    p.nb_state = 99
    h = ctypes.c_void_p()
    rc = lib.dll.cacto_sys_create(ctypes.byref(p), None, ctypes.byref(h))
    assert rc == -1
    assert b"nb_state" in lib.dll.cacto_last_error()


def test_workspace_query_without_gpu_needs_a_handle():
    assert L.lib().dll.cacto_workspace_bytes(None, 128) == 0


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout not present")
@pytest.mark.parametrize("urdf,name", [("double_integrator.urdf", "double_integrator"),
                                       ("planar_manipulator_3dof.urdf", "planar_manipulator_3dof"),
                                       ("ur5_robot.urdf", "ur5")])
def test_builtin_models_match_reference_urdf(urdf, name):
    m = parse_urdf(os.path.join(REFERENCE, "urdf", urdf))
    b = builtin_model(name)
    np.testing.assert_allclose(m.table(), b.table(), atol=1e-12)
    assert m.ee_parent == b.ee_parent
    np.testing.assert_allclose(m.ee_p, b.ee_p)
    np.testing.assert_allclose(m.ee_R, b.ee_R)


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout not present")
def test_ur5_urdf_parses():
    m = parse_urdf(os.path.join(REFERENCE, "urdf", "ur5_robot.urdf"))
    assert m.nq == 6 and m.ee_parent == 5
    assert all(j.kind == 0 for j in m.joints)


def _ref_constants(fname):
    """Literal module-level constants of a reference conf file (read as text, via ast)."""
    import ast
    src = open(os.path.join(REFERENCE, fname)).read()
    out = {}
    for node in ast.parse(src).body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            try:
                out[node.targets[0].id] = ast.literal_eval(node.value)
            except Exception:
                pass
    return out


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout not present")
@pytest.mark.parametrize("system", ["single_integrator", "double_integrator", "manipulator", "car", "car_park", "ur5"])
def test_conf_constants_match_reference(system):
    ref = _ref_constants("conf_%s.py" % system)
    conf = load_conf(system)
    keys = [k for k in ref if hasattr(conf, k) and not k.endswith("_path") and k not in ("test_set",)]
    assert len(keys) > 30
    for k in keys:
        v = getattr(conf, k)
        if isinstance(ref[k], (int, float)) and not isinstance(ref[k], bool):
            assert float(v) == float(ref[k]), k
        elif isinstance(ref[k], str):
            assert v == ref[k], k
