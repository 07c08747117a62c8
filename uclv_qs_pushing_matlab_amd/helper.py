"""helper.closed_loop_matlab mirror (helper.m:195-322), batched and device-resident.

The whole loop runs on the GPU through qsp_closed_loop_ex, one host round trip per call:
the disturbance branch (:221-236: y offset, contact re-projected onto the contour -- MATLAB's
fminunc restated as a damped Newton iteration), sim_noise (:240-242), the controller's delay
prediction delay_buffer_sim and its input buffer (NMPC_controller.m:112-120, helper.m:255),
NMPC_controller.solve, and the plant step with evalModelVariableShape and the plant's own delay
buffer (:289-307).  Not reproduced: print/debug_cost (MATLAB figures and console output).
"""
import numpy as np


def closed_loop_matlab(plant, controller, x0, time_sim, print_=False, sim_noise=False, debug_cost=False,
                       disturbance_=False, amplitude_dist=0.0, t_dist=0, seed=0):
    """Returns (x_s, x_sim, y_s, theta_s, S_p_x, S_p_y, u_n, u_t, time_sim_vec, mode_vect, found_sol),
    each with a leading batch dimension B (helper.m:195-197; x_sim is (B, 2T+1, 4): the reference's
    4 x (2T+1) with its T+1 leading zero columns); amplitude_dist may be per lane."""
    Ts = controller.sample_time
    time_sim_vec = np.arange(0.0, time_sim + 1e-9, Ts)                      # :198
    T = len(time_sim_vec)
    B = controller.batch
    noise = None
    if sim_noise:                                                           # :243-245
        rng = np.random.default_rng(seed)
        noise = rng.standard_normal((T, B, 4)) * np.array([1e-5, 1e-5, 1e-3, 1e-4])
    x0 = np.broadcast_to(np.asarray(x0, np.float64).reshape(-1, 4), (B, 4))
    r = controller.ocp_solver.closed_loop(x0, T, index0=1, noise=noise, plant_delay=plant.time_delay,
                                          disturbance=bool(disturbance_), t_dist=int(t_dist),
                                          amplitude=amplitude_dist)
    X, U = r["X"][:, :T], r["U"]
    found_sol = r["status"] == 0                                            # :253-260
    S_p = plant.SP.FC(X[:, :, 3].ravel()).reshape(B, T, 2)                 # :316-318
    mode_vect = np.zeros((B, T), dtype="<U1")
    # x_sim = [zeros(nx, T+1) xk_sim ...] (helper.m:203, :247): T + 1 zero columns, then one per step
    x_sim = np.concatenate([np.zeros((B, T + 1, 4)), r["Xsim"]], 1)
    return (X[:, :, 0], x_sim, X[:, :, 1], X[:, :, 2], S_p[..., 0], S_p[..., 1], U[:, :, 0], U[:, :, 1],
            time_sim_vec, mode_vect, found_sol)
