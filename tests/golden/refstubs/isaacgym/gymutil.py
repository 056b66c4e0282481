"""gymutil stand-ins: sim-config parsing and device-string parsing."""


def parse_device_str(s):
    if ":" in s:
        t, i = s.split(":")
        return t, int(i)
    return s, 0


def parse_sim_config(cfg, sim_params):
    for k, v in cfg.items():
        if isinstance(v, type) or k.startswith("_"):
            continue
        setattr(sim_params, k, v)


class WireframeSphereGeometry:
    def __init__(self, *a, **k):
        pass


def draw_lines(*a, **k):
    pass
