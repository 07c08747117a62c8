classdef NMPC_controller_hip < handle
    % Drop-in for acados_nmpc/NMPC_controller.m backed by the MI355X library (qsp_nmpc_mex).
    % Same constructor/method names as the reference (NMPC_controller.m:68-431); every per-lane
    % array gains a trailing batch dimension B (B = 1 reproduces it).  The solver options default
    % to create_ocp_opts (:270-300): 'sqp' + merit backtracking, max_iter 30, tol 1e-6.
    properties
        name; plant; sample_time; Hp; T; B
        W_x = 0.01*diag([100 100 0.1 0]); W_x_e = 200*diag([1000 1000 0.1 0]); W_u = diag([1e-3 1e-3])
        u_n_ub = 0.03; u_t_ub = 0.05; u_n_lb = 0; u_t_lb = -0.05
        v_alpha = 0.002*500; d_v_bound = 0; t_angle0 = 3
        delay_compensation = 0; delay_buff_comp = 0
        y_ref = []; cost_function_vect = []
        ocp_opts                      % struct of acados_ocp_opts fields passed to 'create'
        h                             % uint64 library handle
    end
    methods
        function self = NMPC_controller_hip(name, plant, sample_time, Hp, B)
            if nargin < 5, B = 1; end
            self.name = name; self.plant = plant; self.sample_time = sample_time;
            self.Hp = Hp; self.T = Hp*sample_time; self.B = B;
            self.ocp_opts = struct('nlp_solver_type', 'SQP', 'nlp_solver_max_iter', 30, ...
                'nlp_solver_tol_stat', 1e-6, 'nlp_solver_tol_eq', 1e-6, 'nlp_solver_tol_ineq', 1e-6, ...
                'nlp_solver_tol_comp', 1e-6, 'qp_solver_cond_N', 5);           % NMPC_controller.m:271-276
        end
        function create_ocp_solver(self, shapes, shape_id)                  % :302-305
            % shapes: n x 7 cell {ply_path, flip, mu_sg, mu_sp, m, tau_max, xwidth}; shape_id: 1 x B (0-based)
            self.h = qsp_nmpc_mex('create', self.Hp, self.B, self.sample_time, self.ocp_opts);
            qsp_nmpc_mex('shape_ply', self.h, shapes, shape_id);
            qsp_nmpc_mex('cost_W', self.h, [diag(self.W_x); diag(self.W_u)], diag(self.W_x_e));
            qsp_nmpc_mex('constr_h', self.h, [-0.06 self.u_n_lb self.u_t_lb], [0.011 self.u_n_ub self.u_t_ub]);
            qsp_nmpc_mex('ctrl_params', self.h, self.v_alpha, self.d_v_bound, self.t_angle0, self.u_n_lb, self.u_t_ub);
        end
        function update_cost_function(self, W_x, W_u, W_x_e, ~, ~)          % :153-164 (same W on all stages)
            self.W_x = W_x; self.W_u = W_u; self.W_x_e = W_x_e;
            qsp_nmpc_mex('cost_W', self.h, [diag(W_x); diag(W_u)], diag(W_x_e));
        end
        function update_constraints(self, u_n_ub, u_t_ub, u_n_lb, u_t_lb)    % :122-142
            self.u_n_ub = u_n_ub; self.u_t_ub = u_t_ub; self.u_n_lb = u_n_lb; self.u_t_lb = u_t_lb;
            qsp_nmpc_mex('constr_h', self.h, [-0.06 u_n_lb u_t_lb], [0.011 u_n_ub u_t_ub]);
            qsp_nmpc_mex('ctrl_params', self.h, self.v_alpha, self.d_v_bound, self.t_angle0, self.u_n_lb, self.u_t_ub);
        end
        function set_delay_comp(self, delay)                                 % :106-110
            self.delay_compensation = delay;
            self.delay_buff_comp = ceil(delay/self.sample_time);
            qsp_nmpc_mex('delay_comp', self.h, delay);                       % zeroes u_buff_contr
        end
        function xk_sim = delay_buffer_sim(self, ~, x)                       % :112-120
            xk_sim = qsp_nmpc_mex('delay_sim', self.h, x);
        end
        function push_u_buffer(self, u)                                      % helper.m:255
            qsp_nmpc_mex('push_u', self.h, u);
        end
        function clear_variables(self)                                       % :144-151
            self.y_ref = []; self.cost_function_vect = [];
            qsp_nmpc_mex('reset', self.h);
        end
        function initial_condition_update(self, x0)                          % :166-172
            qsp_nmpc_mex('set', self.h, 'constr_x0', x0);
            self.clear_variables();
        end
        function set_reference_trajectory(self, y_ref)                       % :425-431 (prefix applied by the library)
            self.y_ref = y_ref;
            qsp_nmpc_mex('reference', self.h, y_ref);
        end
        function set_v_alpha(self, alpha)                                    % :315-317
            self.v_alpha = alpha;
            qsp_nmpc_mex('ctrl_params', self.h, self.v_alpha, self.d_v_bound, self.t_angle0, self.u_n_lb, self.u_t_ub);
        end
        function u = solve(self, x0, index_time)                             % :329-423
            u = qsp_nmpc_mex('controller_solve', self.h, x0, index_time);
            self.cost_function_vect(:, end+1) = qsp_nmpc_mex('get', self.h, 'cost');
        end
        function v = get(self, field, varargin)                              % ocp_solver.get (helper.m:253,264-269)
            v = qsp_nmpc_mex('get', self.h, field, varargin{:});
        end
        function [X, U, status] = closed_loop(self, x0, n_steps, opts)       % helper.m:195-322 on the device
            if nargin < 4, opts = struct(); end
            [X, U, status] = qsp_nmpc_mex('closed_loop', self.h, x0, n_steps, opts);
        end
        function delete(self)
            if ~isempty(self.h), qsp_nmpc_mex('destroy', self.h); end
        end
    end
end
