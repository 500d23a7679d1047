function [y_OL, exitflag] = dms_tracking_solve_gpu(xmeasure, A, B, N, Q, R, P, T, LAMBDA, PSI, ...
                                                   F_x, h_x, F_u, h_u, F_w_N, h_w_N, x_eq, u_eq, delta, options)
%DMS_TRACKING_SOLVE_GPU  Drop-in for the CasADi/IPOPT solve of
%   examples/DMS_tracking_LMPC_casadi.m:163-167 (form F2): returns y_OL = [x_0..x_N; u_0..u_{N-1};
%   theta] in the layout of full(res.x) for the NLP that costfunction / nonlinearconstraints
%   (:223-287) define - a convex QP: delta-weighted running cost, terminal P and T, dynamics
%   x_{k+1} - x_eq = A (x_k - x_eq) + B (u_k - u_eq), boxes F_x / F_u on every stage, the
%   terminal set on [x_N - x_eq; theta].  In DMS_tracking_LMPC_casadi.m replace
%       res = solver('x0',y_init,'lbx',lb,'ubx',ub,'lbg',con_lb,'ubg',con_ub);  y_OL = full(res.x);
%   by
%       y_OL = dms_tracking_solve_gpu(xmeasure,A,B,N,Q,R,P,T,LAMBDA,PSI,F_x,h_x,F_u,h_u, ...
%                                     F_w_N,h_w_N,x_eq,u_eq,delta);
%   xmeasure may hold several states as columns (one column of y_OL each).  The Python shim
%   bqp.TrackingLMPC builds the same structure and is what the tests drive.
persistent Pst key
if nargin < 20, options = struct(); end
n = size(A, 1); m = size(B, 2); p = size(LAMBDA, 2);
k = {A, B, N, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, delta};
if isempty(Pst) || ~isequal(key, k)
    key = k;
    nv = n + m + p;
    Ex = [eye(n), zeros(n, m), -LAMBDA];
    Eu = [zeros(m, n), eye(m), -PSI];
    Et = [zeros(n, n + m), LAMBDA];
    if isscalar(T), T = T * eye(n); end
    W = repmat(2 * delta * (Ex' * Q * Ex + Eu' * R * Eu), 1, 1, N + 1);   % runningcosts :242-246
    W(:, :, N + 1) = 2 * (Ex' * P * Ex + Et' * T * Et);                     % terminalcosts :248-251
    [xlb, xub] = split_box(F_x, h_x, n);
    [ulb, uub] = split_box(F_u, h_u, m);
    XL = -inf(n, N + 1); XU = inf(n, N + 1);
    XL(:, 2:end) = repmat(xlb, 1, N); XU(:, 2:end) = repmat(xub, 1, N);
    Fp = [F_w_N(:, 1:n), zeros(size(F_w_N, 1), m), F_w_N(:, n + 1:end)];
    Pst = struct('N', N, 'nu', m, 'np', p, 'A', A, 'B', B, 'c', zeros(n, 1), 'W', W, ...
                 'xlb', XL, 'xub', XU, 'ulb', repmat(ulb, 1, N), 'uub', repmat(uub, 1, N), ...
                 'Fp', Fp, 'hp', h_w_N(:), 'poly_stage', N);
end
% deviation coordinates x~ = x - x_eq, u~ = u - u_eq
[X, U, theta, ~, exitflag] = ocp_gpu(Pst, xmeasure - x_eq, options);
y_OL = [X + repmat(x_eq, N + 1, 1); U + repmat(u_eq, N, 1); theta];
end

function [lb, ub] = split_box(F, h, n)
lb = -inf(n, 1); ub = inf(n, 1);
for r = 1:size(F, 1)
    j = find(F(r, :));
    if F(r, j) > 0, ub(j) = h(r) / F(r, j); else, lb(j) = h(r) / F(r, j); end
end
end
