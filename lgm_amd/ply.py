"""Minimal PLY vertex I/O (binary little-endian / ascii) for GaussianRenderer.save_ply / load_ply
(core/gs.py:101-190, which uses the external `plyfile`, absent here). Writes exactly what plyfile writes for a
single 'vertex' element of float32 properties, so files interoperate with 3DGS viewers and gui.py."""
from __future__ import annotations

import numpy as np

_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
          "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
          "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def write_ply(path: str, names, data: np.ndarray) -> None:
    data = np.ascontiguousarray(data, dtype="<f4")
    assert data.ndim == 2 and data.shape[1] == len(names)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {data.shape[0]}"]
    header += [f"property float {n}" for n in names]
    header += ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(data.tobytes())


def read_ply(path: str) -> dict:
    """Returns {property name: 1-D numpy array} of the first element (vertices)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii").strip().split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = [tok[1], int(tok[2]), []]
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError("list properties are not supported")
                cur[2].append((tok[2], _TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        name, count, props = elements[0]
        if fmt == "ascii":
            rows = [f.readline().decode("ascii").split() for _ in range(count)]
            arr = np.array(rows, dtype=np.float64).reshape(count, len(props))
            return {p[0]: arr[:, i].astype(p[1]) for i, p in enumerate(props)}
        endian = "<" if fmt == "binary_little_endian" else ">"
        dt = np.dtype([(p[0], endian + p[1]) for p in props])
        rec = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
        return {p[0]: np.asarray(rec[p[0]]).astype(p[1].replace(">", "<")) for p in props}
