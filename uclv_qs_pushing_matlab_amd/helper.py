"""helper.closed_loop_matlab mirror (helper.m:195-322), batched and device-resident.

The whole loop — controller solve, Euler plant step with evalModelVariableShape, optional
sim_noise — runs on the GPU through qsp_closed_loop; one host round trip per call.
Not reproduced: the disturbance branch (:221-236, needs MATLAB's fminunc to re-locate the
contact point; main.m sets t_dist = 15/0.05 = 300 > the 201 steps of its 10 s run, so the
branch never fires there), print/debug_cost (MATLAB figures) and the plant delay buffer
(delay 0 in every reference configuration).
"""
import numpy as np


def closed_loop_matlab(plant, controller, x0, time_sim, print_=False, sim_noise=False, debug_cost=False,
                       disturbance_=False, amplitude_dist=0.0, t_dist=0, seed=0):
    """Returns (x_s, x_sim, y_s, theta_s, S_p_x, S_p_y, u_n, u_t, time_sim_vec, mode_vect, found_sol),
    each with a leading batch dimension B (helper.m:195-197)."""
    if disturbance_:
        raise NotImplementedError("the disturbance branch (helper.m:221-236) relies on MATLAB fminunc")
    if plant.time_delay != 0:
        raise NotImplementedError("plant delay buffer: only time_delay = 0 (main.m:74-75)")
    Ts = controller.sample_time
    time_sim_vec = np.arange(0.0, time_sim + 1e-9, Ts)                      # :198
    T = len(time_sim_vec)
    B = controller.batch
    noise = None
    if sim_noise:                                                           # :243-245
        rng = np.random.default_rng(seed)
        noise = rng.standard_normal((T, B, 4)) * np.array([1e-5, 1e-5, 1e-3, 1e-4])
    x0 = np.broadcast_to(np.asarray(x0, np.float64).reshape(-1, 4), (B, 4))
    r = controller.ocp_solver.closed_loop(x0, T, index0=1 + controller.delay_buff_comp, noise=noise)
    X, U = r["X"][:, :T], r["U"]
    found_sol = r["status"] == 0                                            # :253-260
    S_p = plant.SP.FC(X[:, :, 3].ravel()).reshape(B, T, 2)                 # :316-318
    mode_vect = np.zeros((B, T), dtype="<U1")
    return (X[:, :, 0], X, X[:, :, 1], X[:, :, 2], S_p[..., 0], S_p[..., 1], U[:, :, 0], U[:, :, 1], time_sim_vec,
            mode_vect, found_sol)
