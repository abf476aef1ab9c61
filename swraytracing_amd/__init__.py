"""swraytracing_amd — MI355X-native wave-packet ray tracing (gfx950 HIP).

The qg_flow_ray_trace hot loop of ndefilippis/SWRaytracing (ode_symplectic
over SpectralScheme / interpolate_U / grid_U / g2k / k2g) as hand-written
CDNA4 kernels behind the C ABI in include/swrt.h, with the reference's
MATLAB call surface mirrored in Python.
"""
from ._lib import Context, SwrtError, load
from .integrate import (PacketEnsemble, ode23_packets, ode_symplectic, raytrace_sw, raytrace_xka, rsw_background,
                        step_packet_xka)
from .io import read_field, write_field
from .qg import QGModel, ReceiverLoop, TwoLayerLoop, qg2layersw_raytrace, qgsw_raytrace
from .stored import read_frame, trace_stored
from .scheme import (BUMP_QG, BUMP_SW, DifferenceScheme, FourierScheme, RaytracingScheme, SnapshotPairScheme,
                     SpectralScheme, g2k, grid_U, interpolate, interpolate_U, k2g)

__all__ = [
    "Context", "SwrtError", "load", "PacketEnsemble", "ode23_packets", "ode_symplectic", "raytrace_sw", "raytrace_xka",
    "rsw_background", "step_packet_xka",
    "read_field", "write_field", "QGModel", "ReceiverLoop", "TwoLayerLoop", "qgsw_raytrace", "qg2layersw_raytrace",
    "BUMP_QG", "BUMP_SW", "DifferenceScheme", "FourierScheme", "RaytracingScheme", "SnapshotPairScheme",
    "SpectralScheme", "g2k", "grid_U", "interpolate", "interpolate_U", "k2g", "read_frame", "trace_stored",
]
