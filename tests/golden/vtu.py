"""Stdlib decoder for the reference's mock VTU meshes (zlib-compressed, base64 inline, UInt32 header).

Used only by tests/golden/make_golden.py in the survey/build container, where
/root/reference/tests/mock_vtu/*.vtu exist. The decoded arrays are committed as
tests/golden/cylinder_mesh.npz so nothing on the GPU box reads the reference.
"""
import base64
import struct
import xml.etree.ElementTree as ET
import zlib

import numpy as np

_DT = {
    "Float32": np.float32,
    "Float64": np.float64,
    "Int32": np.int32,
    "Int64": np.int64,
    "UInt8": np.uint8,
}


def _decode(text, dtype):
    text = text.strip()
    # header = 3 + nblocks uint32, base64-encoded on its own
    first = base64.b64decode(text[:8])
    nblocks = struct.unpack("<I", first[:4])[0]
    hlen = 4 * (3 + nblocks)
    henc = 4 * ((hlen + 2) // 3)
    header = struct.unpack("<%dI" % (3 + nblocks), base64.b64decode(text[:henc]))
    csizes = header[3:]
    raw = base64.b64decode(text[henc:])
    out, off = [], 0
    for cs in csizes:
        out.append(zlib.decompress(raw[off : off + cs]))
        off += cs
    return np.frombuffer(b"".join(out), dtype=dtype)


def read_vtu(path):
    root = ET.parse(path).getroot()
    piece = root.find("UnstructuredGrid/Piece")
    arrays = {}
    for da in piece.iter("DataArray"):
        a = _decode(da.text, _DT[da.get("type")])
        ncomp = int(da.get("NumberOfComponents", "1"))
        if ncomp > 1:
            a = a.reshape(-1, ncomp)
        arrays[da.get("Name")] = a.copy()
    return arrays
