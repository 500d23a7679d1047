function [opt_var, exitflag] = tracking_solve_gpu(x, xs, N, K, P, T, LAMBDA, PSI, run_F, run_h, ...
                                                 F_xTheta, f_xTheta, params, options)
%TRACKING_SOLVE_GPU  Drop-in for the fmincon solve of trackingMPC/RunExample.m:134-136 (form F5).
%   Solves the QP of costFunction.m (running cost for k <= N-2 on (x_k - LAMBDA theta, u_k -
%   PSI theta), terminal P on x_{N-1}, offset cost (LAMBDA theta - xs)' T (LAMBDA theta - xs))
%   subject to constraintsFunction.m (run_F [x_k; u_k] <= run_h for k = 0..N-1, terminal set
%   F_xTheta [x_N; theta] <= f_xTheta) with the batched interior-point kernel of libbqp
%   (ocp_gpu MEX).  In RunExample.m replace
%       opt_var = fmincon(COSTFUN,opt_var,[],[],[],[],[],[],CONSFUN,options);
%   by
%       opt_var = tracking_solve_gpu(x,xs,N,K,P,T,LAMBDA,PSI,run_F,run_h,F_xTheta,f_xTheta,params);
%   params: the struct of RunExample.m (A, B, Q, R).  x / xs may hold several states /
%   references as columns (one solve for the batch).  opt_var = [u_0..u_{N-1}; theta] in
%   fmincon's layout.  K is unused (the reference's costFunction takes it but applies u
%   directly).  The Python shim is bqp.TrackingMPC (learning-based-mpc_amd/bqp/mpc.py).
if nargin < 14, options = struct(); end
A = params.A; B = params.B; Q = params.Q; R = params.R;
n = size(A, 1); m = size(B, 2); p = size(LAMBDA, 2);
nv = n + m + p;
% v_k = [x_k; u_k; theta]
Ex = [eye(n), zeros(n, m), -LAMBDA];
Eu = [zeros(m, n), eye(m), -PSI];
Et = [zeros(n, n + m), LAMBDA];
W = zeros(nv, nv, N + 1);
for k = 1:N - 1                                   % costFunction.m: stages 0..N-2
    W(:, :, k) = 2 * (Ex' * Q * Ex + Eu' * R * Eu);
end
W(:, :, N) = W(:, :, N) + 2 * (Ex' * P * Ex);     % terminal P on x_{N-1}
W(:, :, N + 1) = 2 * (Et' * T * Et);              % offset cost on theta
nb = size(x, 2);
if size(xs, 2) == 1, xs = repmat(xs, 1, nb); end
w = zeros(nv, N + 1, nb);
for i = 1:nb
    w(:, N + 1, i) = -2 * Et' * T * xs(:, i);
end
% run_F [x; u] <= run_h: the box rows of |x| <= 5, |u| <= 0.3 as bounds
[lb, ub] = split_box(run_F, run_h, n + m);
XL = repmat(lb(1:n), 1, N + 1); XU = repmat(ub(1:n), 1, N + 1);
XL(:, 1) = -inf; XU(:, 1) = inf;                  % x_0 is fixed (its rows are constants)
XL(:, N + 1) = -inf; XU(:, N + 1) = inf;          % x_N: the terminal set only
UL = repmat(lb(n + 1:end), 1, N); UU = repmat(ub(n + 1:end), 1, N);
Fp = [F_xTheta(:, 1:n), zeros(size(F_xTheta, 1), m), F_xTheta(:, n + 1:end)];   % on [x_N; theta]
Pst = struct('N', N, 'nu', m, 'np', p, 'A', A, 'B', B, 'c', zeros(n, 1), 'W', W, 'w', w, ...
             'xlb', XL, 'xub', XU, 'ulb', UL, 'uub', UU, 'Fp', Fp, 'hp', f_xTheta(:), ...
             'poly_stage', N);
[~, U, theta, ~, exitflag] = ocp_gpu(Pst, x, options);
opt_var = [U; theta];
end

function [lb, ub] = split_box(F, h, nv)
% rows e_j' v <= h or -e_j' v <= h (the reference's run_F layout) -> bounds
lb = -inf(nv, 1); ub = inf(nv, 1);
for r = 1:size(F, 1)
    j = find(F(r, :));
    if numel(j) ~= 1, error('tracking_solve_gpu: run_F row %d is not a box row', r); end
    if F(r, j) > 0, ub(j) = h(r) / F(r, j); else, lb(j) = h(r) / F(r, j); end
end
end
