"""Minimal gymapi surface needed to construct the reference env with a fake gym."""

SIM_PHYSX = 1
SimType = int
DOF_MODE_NONE = 0
DOF_MODE_EFFORT = 3
IMAGE_COLOR = 0
FOLLOW_POSITION = 0
KEY_ESCAPE = 0
KEY_V = 1
UP_AXIS_Z = 1


class _Obj:
    def __init__(self, *a, **k):
        self.__dict__.update(k)

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        v = _Obj()
        object.__setattr__(self, name, v)
        return v


class Vec3(_Obj):
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = x, y, z


class Quat(_Obj):
    def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
        self.x, self.y, self.z, self.w = x, y, z, w

    @staticmethod
    def from_axis_angle(axis, angle):
        return Quat()


class Transform(_Obj):
    def __init__(self, p=None, r=None):
        self.p = p if p is not None else Vec3()
        self.r = r if r is not None else Quat()


class SimParams(_Obj):
    pass


class PlaneParams(_Obj):
    pass


class TriangleMeshParams(_Obj):
    def __init__(self):
        self.transform = Transform()


class AssetOptions(_Obj):
    pass


class CameraProperties(_Obj):
    pass


class RigidShapeProperties(_Obj):
    pass


_FACTORY = None


def acquire_gym():
    if _FACTORY is None:
        raise RuntimeError("fake gym factory not installed (tests/golden/make_golden.py)")
    return _FACTORY()
