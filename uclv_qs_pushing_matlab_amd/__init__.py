"""MI355X-native batched NMPC solver for the quasi-static pusher-slider OCP.

Drop-in for the solver hot path of Vanvitelli-Robotics/uclv_qs_pushing_matlab
(acados_ocp created in acados_nmpc/NMPC_controller.m:302-305): HIP kernels for
gfx950 behind the C ABI in include/qsp_nmpc.h, with Python mirrors of the
reference's NMPC_controller / PusherSliderModel / object_selection interfaces.
"""
from ._lib import QspError, LIB_PATH  # noqa: F401
from .objects import object_selection, make_shape, OBJECT_NAMES  # noqa: F401

__all__ = ["QspError", "object_selection", "make_shape", "OBJECT_NAMES", "OcpSolver", "NMPCController",
           "PusherSliderModel", "TrajectoryGenerator"]


def __getattr__(name):
    if name == "OcpSolver":
        from .solver import OcpSolver
        return OcpSolver
    if name == "NMPCController":
        from .controller import NMPCController
        return NMPCController
    if name == "PusherSliderModel":
        from .model import PusherSliderModel
        return PusherSliderModel
    if name == "TrajectoryGenerator":
        from .trajectory import TrajectoryGenerator
        return TrajectoryGenerator
    raise AttributeError(name)
