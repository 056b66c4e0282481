"""terrain_utils stand-ins: SubTerrain container and a dummy trimesh conversion."""
import numpy as np


class SubTerrain:
    def __init__(self, terrain_name="terrain", width=256, length=256, vertical_scale=1.0, horizontal_scale=1.0):
        self.terrain_name = terrain_name
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.width = width
        self.length = length
        self.height_field_raw = np.zeros((self.width, self.length), dtype=np.int16)


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    return np.zeros((3, 3), dtype=np.float32), np.zeros((1, 3), dtype=np.uint32)


def random_uniform_terrain(*a, **k):
    raise NotImplementedError
