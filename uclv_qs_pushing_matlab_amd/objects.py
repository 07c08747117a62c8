"""Slider database and shape construction.

object_selection mirrors acados_nmpc/objects_database/object_selection.m:1-47; the
contour -> B-spline preprocessing runs in the C ABI (qsp_shape_from_ply,
PusherSliderModel.m:84-132).
"""
import os

from . import _lib

G = 9.81  # helper.m:3
DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

_DB = {
    # object_selection.m:3-42
    "santal": dict(mu_sg=0.32, mu_sp=0.19, xwidth=0.068, ywidth=0.082, m=0.2875, tau_max=0.0251,
                   cad_model_path="cad_santal_centered_scaled_rotated_reduced.stl",
                   pcl_path="planar_surface_santal_36_uniformed.ply"),
    "balea": dict(mu_sg=0.35, mu_sp=0.20, xwidth=0.071, ywidth=0.071, m=0.1713, tau_max=0.0042,
                  cad_model_path="Balea_cad_model v1.stl", pcl_path="Balea_cad_model_planar_surface_36.ply"),
    "montana": dict(mu_sg=0.20, mu_sp=0.10, xwidth=0.057, ywidth=0.101, m=0.2467, tau_max=0.0101,
                    cad_model_path="Montana_cad_model.stl", pcl_path="Montana_cad_model_planar_section_34.ply"),
    "pulirapid": dict(mu_sg=0.22, mu_sp=0.1, xwidth=0.13, ywidth=0.23, m=0.500, tau_max=0.0251,
                      cad_model_path="pulirapid_ricarica_simplified.stl",
                      pcl_path="pulirapid_ricarica_test_curvatura2_ply.ply"),
}
OBJECT_NAMES = tuple(_DB)
# contour orientation flip (PusherSliderModel.m:107-109)
_FLIP = {"santal": 0, "balea": 0, "montana": 1, "pulirapid": 1}


def object_selection(name):
    """Physical parameters of a slider (object_selection.m).  Unknown names raise ValueError
    (the reference prints a message and returns nothing, :43-45)."""
    if name not in _DB:
        raise ValueError(f"Invalid object! Please, chose between: {', '.join(_DB)}")
    d = dict(_DB[name])
    d["area"] = d["xwidth"] * d["ywidth"]
    return d


def make_shape(name, slider=None, pcl_path=None):
    """qsp_shape for a slider: PLY contour -> control points, knots, c_ellipse."""
    slider = slider or object_selection(name)
    path = pcl_path or os.path.join(DATA_DIR, slider["pcl_path"])
    sh = _lib.Shape()
    rc = _lib.lib().qsp_shape_from_ply(path.encode(), _FLIP.get(name, 0), slider["mu_sg"], slider["mu_sp"],
                                       slider["m"], slider["tau_max"], sh)
    _lib.check(rc, "qsp_shape_from_ply")
    sh.xwidth = slider["xwidth"]          # contact re-projection after a disturbance (helper.m:229)
    return sh
