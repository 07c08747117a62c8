"""NMPC_controller mirror (acados_nmpc/NMPC_controller.m), batched over B lanes.

Same method names, argument meaning and defaults as the reference class; every
per-lane quantity gains a leading batch dimension (B = 1 reproduces the reference).
The solver backend is the HIP C ABI (OcpSolver) instead of acados:
  create_ocp_solver        :302-305     acados_ocp(...)        -> OcpSolver
  initial_condition_update :166-172     'constr_x0' + clear_variables
  update_cost_function     :153-164     'cost_W' per stage (diagonal weights)
  update_constraints       :122-142     (unused by main.m; sets u bounds)
  set_reference_trajectory :425-431
  update_tangential_velocity_bounds :319-327
  solve(x0, index_time)    :329-423     s pre-wrap, y_ref staging, warm start, clip,
                                        Euler rollout, SQP, shift, u0 (all on the GPU)
Status follows acados: ocp_solver.get('status') per lane (helper.m:253).
"""
import numpy as np

from .solver import OcpSolver


class NMPCController:
    def __init__(self, name, plant, sample_time, Hp, batch=1, nlp_solver_type="SQP", sqp_iters=30, qp_iters=None,
                 device=0, stages_per_lane=0, qp_solver_cond_N=5):
        # create_ocp_opts (:270-300): 'SQP' with merit backtracking, max_iter 30, tol 1e-6;
        # nlp_solver_type='SQP_RTI' gives the fixed-K full-step iteration of the BASELINE metric.
        # qp_iters: the QP iteration cap -- acados' qp_solver_iter_max default 50 (the reference leaves
        # it) for 'SQP', as the MEX gateway sets it (integration/matlab/qsp_nmpc_mex.c); the library's
        # 20 for the fixed-K 'SQP_RTI' metric
        if qp_iters is None:
            qp_iters = 50 if nlp_solver_type == "SQP" else 20
        self.name = name
        self.plant = plant
        self.sample_time = sample_time
        self.Hp = int(Hp)
        self.T = self.Hp * sample_time                                     # :89
        self.batch = int(batch)
        # properties (:16-26) and ctor constants (:83-84, 98-100)
        self.W_x = 0.01 * np.diag([100, 100, 0.1, 0])
        self.W_x_e = 200 * np.diag([1000, 1000, 0.1, 0])
        self.W_u = np.diag([1e-3, 1e-3])
        self.u_n_ub, self.u_t_ub, self.u_n_lb, self.u_t_lb = 0.03, 0.05, 0.0, -0.05
        self.h_constr_ub = np.array([10, self.u_n_ub, self.u_t_ub])
        self.h_constr_lb = np.array([-10, self.u_n_lb, self.u_t_lb])
        self.v_alpha = 0.002 * 500
        self.d_v_bound = 0.0
        self.t_angle0 = 3.0
        self.delay_compensation = 0.0
        self.delay_buff_comp = 0
        self.initial_condition = np.zeros((self.batch, 4))
        self.y_ref = None
        self.cost_function_vect = []
        # qp_solver_cond_N = 5 as :276 (checked, same QP solution; OcpSolver's note)
        self._opts = dict(nlp_solver_type=nlp_solver_type, sqp_iters=sqp_iters, qp_iters=qp_iters, device=device,
                          stages_per_lane=stages_per_lane, qp_solver_cond_N=min(qp_solver_cond_N, self.Hp))
        self.ocp_solver = None
        self._shape_id = np.zeros(self.batch, np.int32)

    # -------------------------------------------------------------- set-up
    def create_ocp_solver(self, shapes=None, shape_id=None):
        """acados_ocp(create_ocp_model(), create_ocp_opts()) (:302-305).  `shapes` defaults to
        the plant's contour; pass several shapes + shape_id to mix sliders per lane."""
        s = OcpSolver(N=self.Hp, batch=self.batch, Ts=self.sample_time, **self._opts)
        s.set_shapes(shapes if shapes is not None else [self.plant.shape])
        if shape_id is not None:
            self._shape_id = np.broadcast_to(np.asarray(shape_id, np.int32), (self.batch,)).copy()
        s.set_shape_ids(self._shape_id)
        # constraints h = [s; u_n; u_t] with the s-bounds of create_ocp_model (:251-252)
        s.set("constr_lh", [-0.06, self.h_constr_lb[1], self.h_constr_lb[2]])
        s.set("constr_uh", [0.011, self.h_constr_ub[1], self.h_constr_ub[2]])
        s.set("cost_W", np.diag(np.concatenate([np.diag(self.W_x), np.diag(self.W_u)])))
        s.set("cost_W", self.W_x_e, self.Hp)
        self.ocp_solver = s
        self._push_ctrl_params()

    def _push_ctrl_params(self):
        if self.ocp_solver is not None:
            self.ocp_solver.set_ctrl_params(self.v_alpha, self.d_v_bound, self.t_angle0, self.u_n_lb, self.u_t_ub)

    def set_v_alpha(self, alpha):                                          # :315-317
        self.v_alpha = alpha
        self._push_ctrl_params()

    def set_delay_comp(self, delay):                                       # :106-110
        """delay_buff_comp = ceil(delay / Ts); the per-lane input buffer u_buff_contr (device) starts at
        zero; the reference table is read with the delay_buff_comp prefix columns (:425-431)."""
        if self.ocp_solver is None:
            raise RuntimeError("create_ocp_solver before set_delay_comp")
        self.ocp_solver.set_delay_comp(delay)
        self.delay_compensation = float(delay)
        self.delay_buff_comp = self.ocp_solver.delay_cols()

    def delay_buffer_sim(self, plant, x):                                  # :112-120
        """x predicted delay_buff_comp steps ahead with the buffered inputs (oldest first)."""
        return self.ocp_solver.delay_buffer_sim(np.broadcast_to(np.asarray(x, np.float64).reshape(-1, 4),
                                                                (self.batch, 4)))

    def push_u_buffer(self, u):
        """u_buff_contr = [u, u_buff_contr(:, 1:end-1)] -- the update helper.m:255 performs."""
        self.ocp_solver.delay_buffer_push(np.broadcast_to(np.asarray(u, np.float64).reshape(-1, 2), (self.batch, 2)))

    def update_constraints(self, u_n_ub, u_t_ub, u_n_lb, u_t_lb):          # :122-142
        self.u_n_lb, self.u_n_ub, self.u_t_lb, self.u_t_ub = u_n_lb, u_n_ub, u_t_lb, u_t_ub
        self.h_constr_ub = np.array([self.h_constr_ub[0], u_n_ub, u_t_ub])
        self.h_constr_lb = np.array([self.h_constr_lb[0], u_n_lb, u_t_lb])
        if self.ocp_solver is not None:
            self.ocp_solver.set("constr_lh", [-0.06, u_n_lb, u_t_lb])
            self.ocp_solver.set("constr_uh", [0.011, u_n_ub, u_t_ub])
        self._push_ctrl_params()

    def clear_variables(self):                                             # :144-151
        self.y_ref = None
        self.cost_function_vect = []
        if self.ocp_solver is not None:
            self.ocp_solver.controller_reset()

    def update_cost_function(self, W_x, W_u, W_x_e, initial_step, final_step):   # :153-164
        if initial_step != 0 or final_step != self.Hp - 1:
            raise ValueError("per-stage weights are not supported: the same W applies to stages 0..Hp-1")
        W = np.zeros((6, 6))
        W[:4, :4] = W_x
        W[4:, 4:] = W_u
        self.ocp_solver.set("cost_W", np.asarray(W_x_e, np.float64), self.Hp)
        self.ocp_solver.set("cost_W", W)
        self.W_x, self.W_u, self.W_x_e = np.asarray(W_x), np.asarray(W_u), np.asarray(W_x_e)

    def initial_condition_update(self, new_initial_condition):            # :166-172
        x0 = np.asarray(new_initial_condition, np.float64)
        self.initial_condition = np.broadcast_to(x0.reshape(-1, 4), (self.batch, 4)).copy()
        self.ocp_solver.set("constr_x0", self.initial_condition)
        self.clear_variables()

    def set_reference_trajectory(self, y_ref):                            # :425-431
        y = np.asarray(y_ref, np.float64)
        if y.shape[0] != 6:
            raise ValueError("y_ref must be 6 x T ([x; y; theta; s; u_n; u_t] per column)")
        self.y_ref = y
        self.ocp_solver.set_reference_trajectory(y)

    def update_tangential_velocity_bounds(self, s):                       # :319-327
        s = np.asarray(s, np.float64).ravel()
        vb = self.ocp_solver.eval_vbound(s, self._shape_id[:len(s)] if len(s) == self.batch else 0)
        t_angle = np.abs(self.plant.SP.getAngleCurvatures(s)) if self.plant is not None else None
        return vb, t_angle

    # --------------------------------------------------------------- solve
    def solve(self, x0, index_time):
        """u = solve(x0, index_time) (:329-423): x0 is B x 4 (or 4,), index_time 1-based."""
        if self.y_ref is None:
            raise RuntimeError("set_reference_trajectory must be called before solve")
        x0 = np.asarray(x0, np.float64).reshape(-1, 4)
        u = self.ocp_solver.controller_solve(np.broadcast_to(x0, (self.batch, 4)), index_time)
        self.cost_function_vect.append(self.ocp_solver.get_cost())      # :420
        return u
