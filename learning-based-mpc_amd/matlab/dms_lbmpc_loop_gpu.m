function [x, u, xl, exitflag, iterations, data] = dms_lbmpc_loop_gpu(x_init, mpciterations, ...
    delta, N, q, A, B, Q, R, P, T, LAMBDA, PSI, F_x, h_x, F_u, h_u, F_w_N, h_w_N, F_x_d, h_x_d, ...
    x_eq, u_eq, options)
%DMS_LBMPC_LOOP_GPU  Drop-in for the closed loop of examples/DMS_LBMPC_casadi.m:163-218.
%   Per step: the learned-model NLP of the script (cost on the LEARNED states xl, running and
%   terminal, :223-247; nominal states carry the constraints, :254-292) at the measured state,
%   one RK4 plant step (`dynamic`, :297-304) with the first input, get_data.m's update of the
%   8 x q window [X; Y; v] - for a batch of initial states (columns of x_init), all on the GPU
%   (lbmpc_loop_gpu MEX -> bqp_closed_loop_sqp).  Replaces the whole
%       for iter = 1:mpciterations ... solver('x0',y_init,...,'p',data) ... end
%   block; returns x (n x mpciterations+1 x batch), u (m x mpciterations x batch), the learned
%   one-step predictions xl (casadiL2NW.m), the per-step exit flags and SQP iterations, and
%   the final windows (8 x q x batch, ring order).  Warm start: the script's shifted guess
%   (:209-213, Kstabil = 0 tail).  The Python shim is bqp.closed_loop_sqp with bqp.DMSLBMPC.
if nargin < 24, options = struct(); end
n = size(A, 1); m = size(B, 2); p = size(LAMBDA, 2);
nz = N * m + p;
% condensed nominal constraints of each step in deviation coordinates (z = [u - u_eq; theta]):
% F_x_d and the terminal set on [x_1; theta] (:264-270), boxes on x_1..x_N and u_0..u_{N-1}
Sx = cell(N + 1, 1); Mx = cell(N + 1, 1);
Mx{1} = eye(n); Sx{1} = zeros(n, nz);
for k = 1:N
    Eu = zeros(m, nz); Eu(:, (k - 1) * m + (1:m)) = eye(m);
    Mx{k + 1} = A * Mx{k}; Sx{k + 1} = A * Sx{k} + B * Eu;
end
Et = [zeros(p, N * m), eye(p)];
Ain = [F_x_d * Sx{2}; F_w_N(:, 1:n) * Sx{2} + F_w_N(:, n + 1:end) * Et];
b0 = [h_x_d(:); h_w_N(:)];
Bx = [-F_x_d * Mx{2}; -F_w_N(:, 1:n) * Mx{2}];
for k = 1:N
    Eu = zeros(m, nz); Eu(:, (k - 1) * m + (1:m)) = eye(m);
    Ain = [Ain; F_x * Sx{k + 1}; F_u * Eu]; %#ok<AGROW>
    b0 = [b0; h_x(:); h_u(:)]; %#ok<AGROW>
    Bx = [Bx; -F_x * Mx{k + 1}; zeros(size(F_u, 1), n)]; %#ok<AGROW>
end
if isscalar(T), T = T * eye(n); end
Pm = struct('N', N, 'n_run', N, 'term_learned', 1, 'hessian', 1, 'A', A, 'B', B, ...
            'K', zeros(m, n), 'Lq', chol(delta * Q), 'Lr', chol(delta * R), 'Lp', chol(P), ...
            'Lt', chol(T), 'LAMBDA', LAMBDA, 'PSI', PSI, 'xs', zeros(n, 1), 'Ain', Ain, ...
            'bin0', b0, 'Bx', Bx, 'bandwidth', 0.5, 'lambda', 1e-3);
L = struct('steps', mpciterations, 'delta', delta, 'x_eq', x_eq(:), 'u_eq', u_eq(:), 'q', q, ...
           'mask', 1, 'warm', 1);
[X, U, E, XL, I, Wn] = lbmpc_loop_gpu(Pm, L, x_init, options);
nb = size(x_init, 2);
x = reshape(X, n, mpciterations + 1, nb);
u = reshape(U, m, mpciterations, nb);
xl = reshape(XL, n, mpciterations + 1, nb);
exitflag = E; iterations = I;
data = reshape(Wn, 8, q, nb);
end
