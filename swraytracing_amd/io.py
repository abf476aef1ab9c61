"""Frame I/O in the reference's direct-access binary format.

write_field.m:22-49 / read_field.m:37-98: headerless native-endian fp64,
column-major frames appended to `<name>.bin`; a complex field is a real frame
followed by an imaginary frame.  analysis/load_data.m:29-32 reads
packet_time (0-d series), packet_x / packet_k (N x 2 per frame).
"""
from __future__ import annotations

import numpy as np


def write_field(field, fname, frame=1):
    """Append one frame (write_field.m opens with 'a', so `frame` is ignored
    exactly as fseek on an append stream is, write_field.m:31,36)."""
    field = np.asarray(field)
    with open(str(fname) + ".bin", "ab") as fh:
        if np.iscomplexobj(field):
            fh.write(np.asarray(field.real, dtype=np.float64).tobytes(order="F"))
            fh.write(np.asarray(field.imag, dtype=np.float64).tobytes(order="F"))
        else:
            fh.write(np.asarray(field, dtype=np.float64).tobytes(order="F"))


def read_field(fname, nx=1, ny=1, nz=1, frames=None, is_real=None):
    """read_field(file, nx, ny, nz, frmvec): nx == 1 reads the whole 0-d
    series as a 1 x nframes row (read_field.m:68-70); otherwise frames of
    nx x ny x nz, squeezed (read_field.m:72-97).  Spectral fields (nx ==
    2*ny-1, read_field.m:37-41) are read as re/im frame pairs."""
    data = np.fromfile(str(fname) + ".bin", dtype=np.float64)
    if nx == 1:
        return data[None, :]
    if is_real is None:
        is_real = not (nx == 2 * ny - 1)
    per = nx * ny * nz * (1 if is_real else 2)
    nfr = data.size // per
    frames = list(range(1, nfr + 1)) if frames is None else list(np.atleast_1d(frames))
    out = []
    for fr in frames:
        chunk = data[(fr - 1) * per: fr * per]
        if is_real:
            a = chunk.reshape((nx, ny, nz), order="F")
        else:
            h = per // 2
            a = (chunk[:h] + 1j * chunk[h:]).reshape((nx, ny, nz), order="F")
        out.append(a)
    return np.squeeze(np.stack(out, axis=-1))
