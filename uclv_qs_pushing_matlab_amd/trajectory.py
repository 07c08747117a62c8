"""TrajectoryGenerator mirror (acados_nmpc/TrajectoryGenerator.m).

straight_line (:44-79) is fully specified and reproduced.  waypoints_gen (:96-143)
uses MATLAB's Navigation Toolbox `waypointTrajectory` (not reproducible bit-exactly);
here it is the constant-speed piecewise-linear path through the waypoints with the
segment heading as yaw, sampled at the controller rate — exact for the two-waypoint
straight line of main.m:150-164 (config 1).  Rows: [x; y; yaw; s0; 0] (:140).
"""
import numpy as np


class TrajectoryGenerator:
    def __init__(self, T, vel):
        self.sample_time = T
        self.vel = vel
        self.set_plot = False
        self.waypoints_ = None
        self.waypoints_velocities = None

    def set_target(self, x0, xf, t0, tf):
        self.x0 = np.asarray(x0, np.float64).ravel()
        self.xf = np.asarray(xf, np.float64).ravel()
        self.t0 = t0
        self.tf = tf

    def quintic_(self, time):
        tau = np.asarray(time) / self.tf
        return 6 * tau ** 5 - 15 * tau ** 4 + 10 * tau ** 3

    def straight_line(self, auto_angle=False):
        time = np.arange(self.t0, self.tf + 1e-12, self.sample_time)
        n = len(self.x0)
        d = self.xf[:n] - self.x0
        L = np.linalg.norm(d)
        traj = np.zeros((n, len(time)))
        for k, t in enumerate(time):
            s = self.quintic_(t) * L
            traj[:, k] = self.x0 + s * d / L
        if auto_angle:
            tf_angle = self.tf / 2
            time_angle = np.arange(self.t0, tf_angle + 1e-12, self.sample_time)
            ang = np.ones(len(time))
            da = self.xf[2] - self.x0[2]
            for j, t in enumerate(time_angle):
                s = self.quintic_(t) * abs(da)
                ang[j] = self.x0[2] + s * da / abs(da)
            ang[len(time_angle) - 1:] = ang[len(time_angle) - 1]
            traj = np.vstack([traj[:2], ang[None], traj[3:]])
        return time, traj

    def waypoints_gen(self):
        wp = np.asarray(self.waypoints_, np.float64)
        vel = np.broadcast_to(np.asarray(self.waypoints_velocities, np.float64).ravel(), (len(wp) - 1,))
        seg = np.linalg.norm(np.abs(np.diff(wp[:, :2], axis=0)), axis=1)
        times = np.concatenate([[0.0], np.cumsum(seg / vel)])
        t = np.arange(0.0, times[-1] + 1e-9, self.sample_time)
        pos = np.zeros((len(t), 2))
        yaw = np.zeros(len(t))
        for i, tt in enumerate(t):
            k = min(np.searchsorted(times, tt, side="right") - 1, len(seg) - 1)
            a = (tt - times[k]) / (times[k + 1] - times[k])
            pos[i] = wp[k, :2] + a * (wp[k + 1, :2] - wp[k, :2])
            yaw[i] = np.arctan2(wp[k + 1, 1] - wp[k, 1], wp[k + 1, 0] - wp[k, 0])
        s0 = self.x0[3] if hasattr(self, "x0") and len(self.x0) > 3 else 0.0
        traj = np.vstack([pos[:, 0], pos[:, 1], yaw, np.full(len(t), s0), np.zeros(len(t))])
        return t, traj
