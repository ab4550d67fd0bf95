"""System configs — the `--system-id` plugin surface of the reference (main.py:100-115)."""
import importlib
import importlib.util

SYSTEM_MAP = {
    # system_id: (conf module, Environment class name) — main.py:100-107
    'single_integrator': ('conf_single_integrator', 'SingleIntegrator'),
    'double_integrator': ('conf_double_integrator', 'DoubleIntegrator'),
    'car': ('conf_car', 'Car'),
    'car_park': ('conf_car_park', 'CarPark'),
    'manipulator': ('conf_manipulator', 'Manipulator'),
    'ur5': ('conf_ur5', 'UR5'),
}


def load_conf(system_id, fresh=False):
    """The conf module, as main.py:109 imports it (one shared module object). `fresh=True` returns
    a private copy (a new module object executed from the same source) that a caller may modify
    without affecting other users of the conf (benchmarks and tests overriding e.g. BATCH_SIZE)."""
    try:
        mod, _ = SYSTEM_MAP[system_id]
    except KeyError:
        raise KeyError('System {} not found'.format(system_id))
    name = 'cacto_amd.confs.' + mod
    if not fresh:
        return importlib.import_module(name)
    spec = importlib.util.find_spec(name)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m
