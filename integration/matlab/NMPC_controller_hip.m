classdef NMPC_controller_hip < handle
    % Drop-in for acados_nmpc/NMPC_controller.m backed by the MI355X library.
    % Same constructor/method names as the reference (NMPC_controller.m:68-431);
    % every per-lane array gains a trailing batch dimension B (B = 1 reproduces it).
    properties
        name; plant; sample_time; Hp; T; B
        W_x = 0.01*diag([100 100 0.1 0]); W_x_e = 200*diag([1000 1000 0.1 0]); W_u = diag([1e-3 1e-3])
        u_n_ub = 0.03; u_t_ub = 0.05; u_n_lb = 0; u_t_lb = -0.05
        v_alpha = 0.002*500; d_v_bound = 0; t_angle0 = 3
        y_ref = []; cost_function_vect = []
        h   % uint64 library handle
    end
    methods
        function self = NMPC_controller_hip(name, plant, sample_time, Hp, B)
            if nargin < 5, B = 1; end
            self.name = name; self.plant = plant; self.sample_time = sample_time;
            self.Hp = Hp; self.T = Hp*sample_time; self.B = B;
        end
        function create_ocp_solver(self, shapes, shape_id, sqp_iters)       % NMPC_controller.m:302-305
            % shapes: n x 6 cell {ply_path, flip, mu_sg, mu_sp, m, tau_max}; shape_id: 1 x B (0-based)
            if nargin < 4, sqp_iters = 50; end
            self.h = qsp_nmpc_mex('create', self.Hp, self.B, self.sample_time, sqp_iters);
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
            if delay ~= 0
                error('NMPC_controller_hip:delay', 'only delay = 0 is supported (main.m:74-75)');
            end
        end
        function clear_variables(self)                                       % :144-151
            self.y_ref = []; self.cost_function_vect = [];
            qsp_nmpc_mex('reset', self.h);
        end
        function initial_condition_update(self, x0)                          % :166-172
            self.clear_variables();
        end
        function set_reference_trajectory(self, y_ref)                       % :425-431
            self.y_ref = y_ref;
            qsp_nmpc_mex('reference', self.h, y_ref);
        end
        function set_v_alpha(self, alpha)                                    % :315-317
            self.v_alpha = alpha;
            qsp_nmpc_mex('ctrl_params', self.h, self.v_alpha, self.d_v_bound, self.t_angle0, self.u_n_lb, self.u_t_ub);
        end
        function u = solve(self, x0, index_time)                             % :329-423
            u = qsp_nmpc_mex('controller_solve', self.h, x0, index_time);
            self.cost_function_vect(:, end+1) = qsp_nmpc_mex('get', self.h, 'cost', self.B, 1);
        end
        function delete(self)
            if ~isempty(self.h), qsp_nmpc_mex('destroy', self.h); end
        end
    end
end
