"""Extract the Go1 actuator-net weights from the reference's TorchScript archive
WITHOUT executing anything from it (container-only; never run on the GPU box).

Reference: resources/actuator_nets/unitree_go1.pt, loaded by
go1_gym/envs/base/legged_robot_trajectory_tracking.py:1307-1320 with torch.jit.load.
torch.jit.load would compile and run the archive's code, so instead the archive is
read as a zip: `actuator_network/data.pkl` was disassembled with pickletools (text
only) to map storages -> parameters:

    data/0 -> 0.weight (32, 6)   data/1 -> 0.bias (32,)
    data/2 -> 2.weight (32, 32)  data/3 -> 2.bias (32,)
    data/4 -> 4.weight (1, 32)   data/5 -> 4.bias (1,)
    activation modules 1 and 3: act='softsign'  (x / (1 + |x|))

The raw storages are little-endian float32 and are copied verbatim into
legged_tracking_amd/data/actuator_go1.npz (data, not code).
"""
import io
import pickletools
import sys
import zipfile

import numpy as np

SRC = "/root/reference/resources/actuator_nets/unitree_go1.pt"
DST = sys.argv[1] if len(sys.argv) > 1 else "legged_tracking_amd/data/actuator_go1.npz"

LAYOUT = {"w1": ("0", (32, 6)), "b1": ("1", (32,)), "w2": ("2", (32, 32)),
          "b2": ("3", (32,)), "w3": ("4", (1, 32)), "b3": ("5", (1,))}


def main():
    z = zipfile.ZipFile(SRC)
    # confirm the layout from the pickle disassembly (text), never by unpickling
    out = io.StringIO()
    pickletools.dis(io.BytesIO(z.read("actuator_network/data.pkl")), out=out)
    dis = out.getvalue()
    assert "'softsign'" in dis and dis.count("_rebuild_tensor_v2") >= 1
    arrays = {}
    for name, (key, shape) in LAYOUT.items():
        raw = z.read(f"actuator_network/data/{key}")
        a = np.frombuffer(raw, dtype="<f4").reshape(shape).copy()
        arrays[name] = a
    np.savez(DST, **arrays)
    print("wrote", DST, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
