function [opt_var, exitflag, iterations] = lbmpc_solve_gpu(dx, data, opt_var, A, B, Kstabil, ...
                                                          Q, R, P, T, LAMBDA, PSI, m, F_x, h_x, ...
                                                          F_u, h_u, F_w_N, h_w_N, F_x_d, h_x_d, ...
                                                          N, dx_ref, options)
%LBMPC_SOLVE_GPU  Drop-in for the fmincon solve of functions/ocpLBMPC.m:27-31 (form F3).
%   Solves the NLP of costLBMPC.m (learned rollout u = Kstabil x + c with the NW oracle of
%   oracleL2NW.m, running cost for k < N-1, terminal P on the learned x_N) subject to
%   constraintsLBMPC.m (nominal model: the tightened set F_x_d and the robust terminal set on
%   [x_1; theta] at k = 1, boxes on x_1..x_{N-1} and u_0..u_{N-2}) with the batched SQP of
%   libbqp (lbmpc_gpu MEX: Gauss-Newton / exact-Hessian SQP, QP sub-problems on the GPU).
%   In ocpLBMPC.m replace
%       opt_var = fmincon(COSTFUN,opt_var,[],[],[],[],[],[],CONSFUN,options);
%   by
%       opt_var = lbmpc_solve_gpu(dx,data,opt_var,A,B,Kstabil,Q,R,P,T,LAMBDA,PSI,m, ...
%                                 F_x,h_x,F_u,h_u,F_w_N,h_w_N,F_x_d,h_x_d,N,dx_ref);
%   data: the struct {X, Y} of update_data.m (or the 7 x q matrix [X; Y]).  dx may hold several
%   states as columns (one solve for the batch, one column of opt_var each; opt_var then
%   n x batch or n x 1).  The condensed constraints are rebuilt only when the design changes.
%   The Python shim bqp.LBMPC (learning-based-mpc_amd/bqp/lbmpc.py) builds the same data and is
%   what the tests drive; tests/test_mex_gateway.py drives lbmpc_gpu itself.
persistent Pst key
if nargin < 24, options = struct(); end
n = size(A, 1);
k = {A, B, Kstabil, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d, h_x_d, N, dx_ref};
if isempty(Pst) || ~isequal(key, k)
    key = k;
    p = size(LAMBDA, 2);
    nz = N * m + p;
    % nominal closed rollout x_{k+1} = A x_k + B (K x_k + c_k): x_k = Mx{k} x0 + Sx{k} z,
    % u_k = Mu{k} x0 + Su{k} z  (transitionNominal.m)
    Acl = A + B * Kstabil;
    Mx = cell(N + 1, 1); Sx = cell(N + 1, 1); Mu = cell(N, 1); Su = cell(N, 1);
    Mx{1} = eye(n); Sx{1} = zeros(n, nz);
    for kk = 1:N
        Ec = zeros(m, nz); Ec(:, (kk - 1) * m + (1:m)) = eye(m);
        Mu{kk} = Kstabil * Mx{kk}; Su{kk} = Kstabil * Sx{kk} + Ec;
        Mx{kk + 1} = Acl * Mx{kk}; Sx{kk + 1} = A * Sx{kk} + B * Su{kk};
    end
    Et = [zeros(p, N * m), eye(p)];
    Ain = [F_x_d * Sx{2}; F_w_N(:, 1:n) * Sx{2} + F_w_N(:, n + 1:end) * Et];   % constraintsLBMPC.m:27-30
    b0 = [h_x_d(:); h_w_N(:)];
    Bx = [-F_x_d * Mx{2}; -F_w_N(:, 1:n) * Mx{2}];
    for kk = 1:N - 1                                                          % :32-38
        Ain = [Ain; F_x * Sx{kk + 1}; F_u * Su{kk}]; %#ok<AGROW>
        b0 = [b0; h_x(:); h_u(:)]; %#ok<AGROW>
        Bx = [Bx; -F_x * Mx{kk + 1}; -F_u * Mu{kk}]; %#ok<AGROW>
    end
    if isscalar(T), T = T * eye(n); end
    Pst = struct('N', N, 'n_run', max(N - 2, 0), 'term_learned', 1, 'hessian', 1, ...
                 'A', A, 'B', B, 'K', Kstabil, 'Lq', chol(Q), 'Lr', chol(R), 'Lp', chol(P), ...
                 'Lt', chol(T), 'LAMBDA', LAMBDA, 'PSI', PSI, 'xs', dx_ref(:), 'Ain', Ain, ...
                 'bandwidth', 0.5, 'lambda', 1e-3);
    Pst.b0 = b0; Pst.Bx = Bx;
end
if isstruct(data), W = [data.X; data.Y]; else, W = data; end
bin = Pst.b0 + Pst.Bx * dx;              % one column per instance
P = rmfield(Pst, {'b0', 'Bx'});
[opt_var, exitflag, ~, ~, iterations] = lbmpc_gpu(P, dx, W, bin, opt_var, options);
end
