"""Offline stand-in for params_proto==2.10.5 (absent).

Config classes are plain classes whose nested classes are namespaces.
``vars(C)`` returns a NEW dict of the public, non-callable attributes in
definition order (the survey's reading of params_proto's Meta.__dict__).
"""


_TYPE_DICT = type.__dict__["__dict__"]


class Meta(type):
    @property
    def __dict__(cls):
        out = {}
        for k, v in _TYPE_DICT.__get__(cls).items():
            if k.startswith("_") or isinstance(v, (type, staticmethod, classmethod, property)) or callable(v):
                continue
            out[k] = v
        return out


class ParamsProto(metaclass=Meta):
    def __init_subclass__(cls, **kwargs):
        pass


class PrefixProto(ParamsProto):
    pass


def Proto(default=None, **k):
    return default


Flag = Proto
