"""PusherSliderModel mirror (acados_nmpc/PusherSliderModel.m).

The constructor follows PusherSliderModel.m:45-60 (f_max, c_ellipse, spline from the
PLY contour, :113-132); `evalModelVariableShape` (:606-608) evaluates the same f as the
OCP (:503-603) — on the GPU, through the C ABI.  The STL/Delaunay CAD handling
(:62-75) is visual only and not reproduced.
"""
import numpy as np

from . import objects
from .solver import OcpSolver


class SplineShape:
    """Numeric view of bspline_shape (bspline_shape.m): FC, FC_dot, R_NT, FC_angle_dot."""

    def __init__(self, shape, evaluator):
        self._shape = shape
        self._ev = evaluator
        self.n = shape.n_ctrl
        self.P = np.array([[shape.ctrl[i][0], shape.ctrl[i][1]] for i in range(self.n)])
        self.S = np.array(shape.knots[:self.n + 4])
        self.p = 3
        self.a = 0.0
        self.b = shape.b

    def _mod(self, s):
        # evalSpline / getAngleCurvatures wrap with MATLAB mod (bspline_shape.m:147,193)
        return np.mod(np.asarray(s, np.float64), self.b)

    def FC(self, s):
        return self._ev.eval_spline(self._mod(s))[0]

    def FC_dot(self, s):
        return self._ev.eval_spline(self._mod(s))[1]

    def getAngleCurvatures(self, s):
        return self._ev.eval_spline(self._mod(s))[3]

    def R_NT(self, s):
        D = self.FC_dot(s)
        t = D / np.linalg.norm(D, axis=1, keepdims=True)
        n = np.stack([t[:, 1], -t[:, 0]], 1)
        return np.stack([n, t], 2)   # columns [n t] (bspline_shape.m:110-111)


class PusherSliderModel:
    nx = 4
    nu = 2

    def __init__(self, name, slider_parameters, time_delay=0.0, cad_model_path=None, order_spline=3,
                 pcl_path=None, object_name="santal"):
        if order_spline != 3:
            raise ValueError("only cubic splines (p = 3, main.m:33) are supported")
        self.name = name
        self.object_name = object_name
        self.slider_params = dict(slider_parameters)
        self.slider_params["f_max"] = self.slider_params["mu_sg"] * self.slider_params["m"] * objects.G   # :53
        self.slider_params["c_ellipse"] = self.slider_params["tau_max"] / self.slider_params["f_max"]       # :55
        self.time_delay = time_delay
        self.shape = objects.make_shape(object_name, self.slider_params, pcl_path)
        self._ev = OcpSolver(N=1, batch=1)
        self._ev.set_shapes([self.shape])
        self.SP = SplineShape(self.shape, self._ev)

    def set_delay(self, time_delay):
        self.time_delay = time_delay

    def evalModelVariableShape(self, x, u):
        """x_dot = f(x, u) (PusherSliderModel.m:606-608); batched over leading dimensions."""
        x = np.asarray(x, np.float64)
        u = np.asarray(u, np.float64)
        f, _ = self._ev.eval_dynamics(x.reshape(-1, 4), u.reshape(-1, 2))
        return f.reshape(x.shape)

    def jacobian(self, x, u):
        """d f / d(x, u) (4 x 6 per point) — what CasADi's VDE would differentiate."""
        return self._ev.eval_dynamics(np.reshape(x, (-1, 4)), np.reshape(u, (-1, 2)))[1]
