"""System configs — the `--system-id` plugin surface of the reference (main.py:100-115)."""
import importlib

SYSTEM_MAP = {
    # system_id: (conf module, Environment class name) — main.py:100-107
    'single_integrator': ('conf_single_integrator', 'SingleIntegrator'),
    'double_integrator': ('conf_double_integrator', 'DoubleIntegrator'),
    'car': ('conf_car', 'Car'),
    'car_park': ('conf_car_park', 'CarPark'),
    'manipulator': ('conf_manipulator', 'Manipulator'),
    'ur5': ('conf_ur5', 'UR5'),
}


def load_conf(system_id):
    try:
        mod, _ = SYSTEM_MAP[system_id]
    except KeyError:
        raise KeyError('System {} not found'.format(system_id))
    return importlib.import_module('cacto_amd.confs.' + mod)
