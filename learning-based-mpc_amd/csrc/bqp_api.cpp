// bqp_api.cpp — implementation of the C ABI declared in include/bqp.h.
//
// Host-side responsibilities only: argument validation, workspace management (grow-only device
// buffers owned by the handle), host<->device staging for the host-pointer entry points, and
// dispatch of the HIP kernels (bqp_ocp.hip, bqp_dense.hip, bqp_prep.hip).  No arithmetic of
// the solve happens on the host: there is no CPU fallback path.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/bqp.h"
#include "bqp_internal.h"

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct bqp_handle_s {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    int launches = 0;
    DevBuf work;   // tables + stats (device entry points)
    DevBuf stage;  // staging of host-pointer calls
    DevBuf dwork;  // dense per-instance scratch
    DevBuf lwork;  // learning-based MPC (SQP) buffers
    DevBuf cwork;  // closed-loop simulation buffers
    DevBuf hwork;  // mixed precision: fp32 -> fp64 handoff records
    DevBuf pwork;  // long-horizon layout: global Riccati tables
    DevBuf wwork;  // per-instance stage-cost tables
    int last_batch = 0;
    int* mixed_flags = nullptr;   // the last mixed-mode solve's fp32-phase flags
    int* mixed_cont = nullptr;    // and its continuation's exit flags (bqp_debug_mixed_flags)
    int mixed_batch = 0;
};

namespace {

struct DevScope {
    int prev = -1;
    explicit DevScope(int d) {
        hipGetDevice(&prev);
        if (prev != d) hipSetDevice(d);
    }
    ~DevScope() {
        int cur = -1;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};

inline size_t span(int batch, int64_t stride, size_t n) {
    return n == 0 ? 0 : (size_t)(batch - 1) * (size_t)stride + n;
}

void resolve(const bqp_options* in, bqp_options* o) {
    bqp_default_options(o);
    if (!in) return;
    if (in->max_iter > 0) o->max_iter = in->max_iter;
    if (in->tol_stat > 0) o->tol_stat = in->tol_stat;
    if (in->tol_feas > 0) o->tol_feas = in->tol_feas;
    if (in->tol_comp > 0) o->tol_comp = in->tol_comp;
    if (in->tau > 0 && in->tau < 1) o->tau = in->tau;
    o->precision = in->precision;
    o->want_duals = in->want_duals;
    o->polish = in->polish;
}

#define HIP_TRY(x)                                                        \
    do {                                                                  \
        hipError_t _e = (x);                                              \
        if (_e != hipSuccess) {                                           \
            fprintf(stderr, "bqp: %s failed: %s\n", #x, hipGetErrorString(_e)); \
            return BQP_E_HIP;                                             \
        }                                                                 \
    } while (0)

// an event owned by an entry point's scope: destroyed on every return (HIP_TRY included)
struct EventGuard {
    hipEvent_t e = nullptr;
    ~EventGuard() { if (e) hipEventDestroy(e); }
};

}  // namespace

extern "C" {

const char* bqp_version(void) { return "bqp 0.1.0 (gfx950, structured Riccati Mehrotra IPM)"; }

#ifndef BQP_SRC_SHA1
#define BQP_SRC_SHA1 "unknown"
#endif
const char* bqp_build_source_sha1(void) { return BQP_SRC_SHA1; }

void bqp_default_options(bqp_options* o) {
    if (!o) return;
    o->max_iter = 50;
    o->tol_stat = 1e-8;
    o->tol_feas = 1e-10;
    o->tol_comp = 1e-14;
    o->tau = 0.995;
    o->precision = 0;
    o->want_duals = 0;
    o->polish = 0;
}

int bqp_create(bqp_handle* h, int device) {
    if (!h) return BQP_E_ARG;
    *h = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return BQP_E_NODEV;
    int dev = device;
    if (dev < 0) hipGetDevice(&dev);
    if (dev >= n) return BQP_E_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return BQP_E_NODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "bqp: device %d is %s; this build targets gfx950 only\n", dev, prop.gcnArchName);
        return BQP_E_NODEV;
    }
    bqp_handle_s* s = new bqp_handle_s();
    s->device = dev;
    DevScope ds(dev);
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess) {
        delete s;
        return BQP_E_HIP;
    }
    *h = s;
    return BQP_OK;
}

int bqp_destroy(bqp_handle h) {
    if (!h) return BQP_OK;
    {
        DevScope ds(h->device);
        if (h->stream) hipStreamSynchronize(h->stream);
        h->work.release();
        h->stage.release();
        h->dwork.release();
        h->lwork.release();
        h->cwork.release();
        h->hwork.release();
        h->pwork.release();
        h->wwork.release();
        if (h->ev0) hipEventDestroy(h->ev0);
        if (h->ev1) hipEventDestroy(h->ev1);
        if (h->stream) hipStreamDestroy(h->stream);
    }
    delete h;
    return BQP_OK;
}

int bqp_debug_mixed_flags(bqp_handle h, int batch, int* flags) {
    if (!h || !flags || batch <= 0) return BQP_E_ARG;
    if (!h->mixed_flags || batch != h->mixed_batch) return BQP_E_ARG;
    DevScope ds(h->device);
    HIP_TRY(hipDeviceSynchronize());
    std::vector<int> f2((size_t)2 * batch);
    HIP_TRY(hipMemcpy(f2.data(), h->mixed_flags, sizeof(int) * batch, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(f2.data() + batch, h->mixed_cont, sizeof(int) * batch, hipMemcpyDeviceToHost));
    // the retry launch solved again the instances whose continuation ended != 1 after a warm
    // start (fp32-phase flag 0 / 1): reported as 2
    for (int i = 0; i < batch; ++i) {
        const int hf = f2[i], c2 = f2[(size_t)batch + i];
        flags[i] = ((hf == 0 || hf == 1) && c2 != 1) ? 2 : hf;
    }
    return BQP_OK;
}

int bqp_last_kernel_ms(bqp_handle h, double* ms, int* launches) {
    if (!h || !ms) return BQP_E_ARG;
    *ms = 0.0;
    if (launches) *launches = h->launches;
    if (!h->timed) return BQP_OK;
    DevScope ds(h->device);
    HIP_TRY(hipEventSynchronize(h->ev1));
    float f = 0.f;
    HIP_TRY(hipEventElapsedTime(&f, h->ev0, h->ev1));
    *ms = (double)f;
    return BQP_OK;
}

// ------------------------------------------------------------------------------------------
// structured OCP
// ------------------------------------------------------------------------------------------
static int ocp_check(const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D) {
    if (!d || !D || batch <= 0) return BQP_E_ARG;
    if (d->nx <= 0 || d->nu <= 0 || d->np <= 0 || d->N < 1 || d->n_poly < 0) return BQP_E_ARG;
    if (d->poly_stage < 0 || d->poly_stage > d->N) return BQP_E_ARG;
    if (!D->A || !D->B || !D->W || !D->x0) return BQP_E_ARG;
    if (d->n_poly > 0 && (!D->Fp || !D->hp)) return BQP_E_ARG;
    if (!bqp::ocp_supported(d->nx, d->nu, d->np)) return BQP_E_UNSUPPORTED;
    if (d->N > 127 || bqp::ocp_rpl_for(std::max(d->n_poly, 1)) < 0) return BQP_E_UNSUPPORTED;
    if (D->sW != 0 && D->sW < (int64_t)(d->N + 1) * (d->nx + d->nu + d->np) * (d->nx + d->nu + d->np))
        return BQP_E_ARG;                                     // per-instance stage costs overlap
    if (D->sFp != 0 && D->sFp < (int64_t)d->n_poly * (d->nx + d->nu + d->np)) return BQP_E_ARG;
    return BQP_OK;
}

int bqp_solve_ocp_batched_device(bqp_handle h, const bqp_ocp_dims* d, int batch,
                                 const bqp_ocp_data* D, const bqp_options* opt, double* x,
                                 double* u, double* theta, double* fval, int* exitflag,
                                 bqp_output* out, const bqp_ocp_duals* duals, void* stream) {
    if (!h) return BQP_E_ARG;
    int rc = ocp_check(d, batch, D);
    if (rc) return rc;
    if (!x || !u || !theta || !exitflag) return BQP_E_ARG;
    DevScope ds(h->device);
    hipStream_t st = (hipStream_t)stream;
    bqp_options o;
    resolve(opt, &o);
    if (o.precision < 0 || o.precision > 2) return BQP_E_ARG;
    const bool f32 = o.precision == 1;     // fp32 instantiation (bqp_ocp_f32.hip)
    // fp32 phase, then fp64 from the fp32 iterate; long horizons only (N + 1 > 64, the
    // instantiations that carry the handoff): shorter ones are solved in fp64 alone
    const bool mixed = o.precision == 2 && d->N + 1 > 64;
    bqp_options o32 = o;
    // fp32 arithmetic cannot resolve the fp64 defaults: floor the stopping tolerances
    o32.tol_stat = std::max(o.tol_stat, 1e-5);
    o32.tol_feas = std::max(o.tol_feas, 1e-6);
    o32.tol_comp = std::max(o.tol_comp, 1e-9);
    if (mixed) {
        // hand over once the fp32 iterate is feasible to 1e-6 and mu <= 1e-6: the fp64 launch then
        // needs ~4 iterations and ends at the fp64 solve's KKT accuracy (duals within ~3e-8 of
        // lambda*); later switches (mu 1e-7 .. 1e-9) save 3-7 % of the time but leave the duals
        // of some instances at 1e-7 .. 2e-7 (tools/diag_mixed.py, profiles/r02_mx/diag_switch.log).
        // BQP_MIXED_MU overrides, for that sweep (values outside (0, 1e-3] are ignored).
        o32.tol_comp = std::max(o.tol_comp, 1e-6);
        if (const char* e = getenv("BQP_MIXED_MU")) {
            char* end = nullptr;
            const double v = strtod(e, &end);
            if (end != e && *end == '\0' && v > 0.0 && v <= 1e-3) o32.tol_comp = v;
        }
    }
    if (f32) o = o32;
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N;
    const int nv = nx + nu + np;
    const int mp = d->n_poly;
    const int hstride = nv * nv + 1;
    const int mpad = 64 * bqp::ocp_rpl_for(std::max(mp, 1));   // = the kernel's RPL * 64
    // per-instance polytope (sFp != 0): each instance's LDS slot holds its own NV x mpad table
    const bool fpi = mp > 0 && D->sFp != 0;
    const bool hinst = D->sW != 0;        // per-instance stage costs (the instance's H table)
    // long horizons (two stages per lane): H read from global, Riccati tables in global scratch,
    // polytope rhs / box bounds in the shared tables when the batch shares them (QpLds lng)
    // (fp64 instantiation only; the fp32 one keeps the plain layout)
    struct Shared { bool lng, hpsh, bndsh; int sh_F, sh_hp, sh_bnd, doubles; };
    auto shared_layout = [&](bool single) {
        Shared o;
        o.lng = !single && N + 1 > 64;
        o.hpsh = mp > 0 && D->shp == 0;       // the shared polytope rhs (every horizon)
        o.bndsh = o.lng && D->sxb == 0 && D->sub == 0;
        const int nbr = (N + 1) * 2 * (nx + nu);
        int sh = (o.lng || hinst) ? 0 : (N + 1) * hstride;
        o.sh_F = sh;
        sh += fpi ? 0 : nv * mpad;
        o.sh_hp = o.hpsh ? sh : -1;
        sh += o.hpsh ? mpad : 0;
        o.sh_bnd = o.bndsh ? sh : -1;
        sh += o.bndsh ? nbr : 0;
        o.doubles = (sh + 1) & ~1;   // elements
        return o;
    };
    const Shared L64 = shared_layout(f32), L32 = shared_layout(true);
    const bool lng = L64.lng;
    // instances per workgroup (two waves each) that fit the 160 KB of LDS
    auto fit_wpb = [&](bool single, int& wpb) -> bool {
        const Shared& S = single ? L32 : L64;
        const int shared_doubles = S.doubles;
        const int per_wave = single ? bqp::ocp_wave_lds_doubles_f32(N, nx, nu, np, mpad, fpi, false, S.hpsh, false, hinst)
                                    : bqp::ocp_wave_lds_doubles(N, nx, nu, np, mpad, fpi, S.lng, S.hpsh, S.bndsh, hinst);
        // 160 KB per workgroup less the repair kernel's 256 B of static LDS (its
        // __syncthreads_or scratch): N = 50 at two instances per workgroup sits exactly there
        const size_t lds_budget = (160 * 1024 - 256) / (single ? sizeof(float) : sizeof(double));
        // long horizons (N + 1 > 64, two stages per lane) are compiled for <= 256 threads per
        // workgroup: one wave per SIMD, whose 512 registers hold the doubled stage state
        wpb = (N + 1 > 64) ? 2 : 4;
        // diagnostic (the A/B variants of tools/gpu_r06_*.sh): BQP_OCP_WPB sets the instances per
        // workgroup the LDS budget then caps
        if (const char* e = getenv("BQP_OCP_WPB")) {
            const int v = atoi(e);
            if (v >= 1 && v <= 8) wpb = v;
        }
        while (wpb > 1 && (size_t)shared_doubles + (size_t)wpb * per_wave > lds_budget) --wpb;
        return (size_t)shared_doubles + (size_t)per_wave <= lds_budget;
    };
    int wpb = 1, wpb32 = 1;
    if (!fit_wpb(f32, wpb)) return BQP_E_UNSUPPORTED;
    if (mixed && !fit_wpb(true, wpb32)) return BQP_E_UNSUPPORTED;
    // workspace: H, Fp, stats
    const size_t nH = (size_t)(N + 1) * hstride, nF = (size_t)nv * mpad, nS = (size_t)batch * bqp::STATS_W;
    // + the repair marks (one int per instance, after the stamps of the diagnostic build)
    const size_t nPol = ((size_t)batch + 1) / 2;
#ifdef BQP_STAMPS
    const size_t nStamp = (size_t)batch * 32;
#else
    const size_t nStamp = 0;
#endif
    // + the work-queue counters of the launches (bqp::OCP_QUEUES ints)
    const size_t nQ = (bqp::OCP_QUEUES + 1) / 2;
    HIP_TRY(h->work.reserve(sizeof(double) * (nH + nF + nS + 8 + nStamp + nPol + nQ)));
    double* Hd = (double*)h->work.p;
    double* Fd = Hd + nH;
    double* Sd = Fd + nF;
    int* polneed = (int*)(Sd + nS + 8 + nStamp);
    int* queues = (int*)(Sd + nS + 8 + nStamp + nPol);
    const double* Hinst = nullptr;
    if (hinst) {   // per-instance prepared stage-cost tables
        HIP_TRY(h->wwork.reserve(sizeof(double) * (size_t)batch * nH));
        HIP_TRY(bqp::launch_ocp_prep_h(D->W, D->sW, batch, nx, nu, np, N, hstride, (double*)h->wwork.p, st));
        Hinst = (const double*)h->wwork.p;
    }
    void* Pg = nullptr;
    if (lng) {   // global Riccati tables of the long-horizon layout
        HIP_TRY(h->pwork.reserve(sizeof(double) * (size_t)batch * (N + 1) * bqp::ocp_pstride(nx + np)));
        Pg = h->pwork.p;
    }
    HIP_TRY(bqp::launch_ocp_prep(D->W, mp > 0 ? D->Fp : D->W, nx, nu, np, N, mp, d->poly_stage,
                                 hstride, mpad, Hd, Fd, queues, st));
    bqp::OcpKernelArgs a;
    memset(&a, 0, sizeof(a));
    // the solve launch's work queue (used when the batch exceeds the resident workgroups)
    a.queue = queues;
    a.N = N; a.mp = mp; a.kp = d->poly_stage; a.batch = batch; a.wpb = wpb;
    const Shared& LS = f32 ? L32 : L64;
    a.hstride = hstride; a.mpad = mpad; a.shared_doubles = LS.doubles;
    a.Pg = Pg; a.sh_F = LS.sh_F; a.sh_hp = LS.sh_hp; a.sh_bnd = LS.sh_bnd; a.H_inst = Hinst;
    a.max_iter = o.max_iter; a.tol_stat = o.tol_stat; a.tol_feas = o.tol_feas;
    a.tol_comp = o.tol_comp; a.tau = o.tau;
    a.polish = o.polish < 0 ? 0 : (o.polish == 0 ? 1 : std::min(o.polish, 2));
    a.pol_need = polneed;
    a.H = Hd; a.Fp = Fd;
    a.A = D->A; a.B = D->B; a.c = D->c; a.w = D->w; a.xlb = D->xlb; a.xub = D->xub;
    a.ulb = D->ulb; a.uub = D->uub; a.hp = mp > 0 ? D->hp : Hd; a.x0 = D->x0;
    a.sA = D->sA; a.sB = D->sB; a.sc = D->sc; a.sw = D->sw; a.sxb = D->sxb; a.sub = D->sub;
    a.shp = D->shp; a.sx0 = D->sx0;
    if (fpi) { a.Fp_inst = D->Fp; a.sFp = D->sFp; }
    a.x = x; a.u = u; a.theta = theta; a.fval = fval; a.exitflag = exitflag; a.stats = Sd;
    if (duals) {
        a.pi_out = duals->pi; a.lamx_out = duals->lam_x; a.lamu_out = duals->lam_u;
        a.lamp_out = duals->lam_p;
    }
#ifdef BQP_STAMPS
    a.stamps = Sd + nS + 8;
    h->last_batch = batch;
#endif
    HIP_TRY(hipEventRecord(h->ev0, st));
    if (mixed) {
        // phase 1: fp32 to the floored tolerances, iterate to the handoff records
        const int hf = bqp::ocp_hand_floats(N, nx, nu, np, mp);
        if (hf <= 0) return BQP_E_UNSUPPORTED;
        const size_t hrec = ((size_t)hf + 63) & ~(size_t)63;
        HIP_TRY(h->hwork.reserve(sizeof(float) * hrec * batch + 3 * sizeof(int) * (size_t)batch));
        float* hb = (float*)h->hwork.p;
        int* hflag = (int*)(hb + hrec * batch);
        int* hit = hflag + batch;
        int* c2flag = hit + batch;    // the continuation's exit flags (diagnostic)
        h->mixed_flags = hflag;
        h->mixed_cont = c2flag;
        h->mixed_batch = batch;
        bqp::OcpKernelArgs a1 = a;
        a1.wpb = wpb32;
        a1.shared_doubles = L32.doubles; a1.sh_F = L32.sh_F; a1.sh_hp = L32.sh_hp; a1.sh_bnd = L32.sh_bnd;
        a1.max_iter = o32.max_iter; a1.tol_stat = o32.tol_stat; a1.tol_feas = o32.tol_feas;
        a1.tol_comp = o32.tol_comp;
        a1.exitflag = hflag;
        a1.hand_out = hb; a1.hand_it = hit; a1.hand_stride = (int64_t)hrec;
        a1.pi_out = a1.lamx_out = a1.lamu_out = a1.lamp_out = nullptr;
        a1.queue = queues + 1;
        HIP_TRY(bqp::launch_ocp_f32(a1, nx, nu, np, st));
        // phase 2: fp64 from the handed-over iterates
        a.hand_in = hb; a.hand_flag = hflag; a.hand_it = hit; a.hand_stride = (int64_t)hrec;
        HIP_TRY(bqp::launch_ocp(a, nx, nu, np, st));
        // (diagnostic record of the continuation's exit flags, for bqp_debug_mixed_flags)
        HIP_TRY(hipMemcpyAsync(c2flag, exitflag, sizeof(int) * batch, hipMemcpyDeviceToDevice, st));
        // phase 3: a continuation that did not converge (-8 / -2 / 0: marginal instances, e.g.
        // nearly infeasible perturbed models) is solved again from the fp64 initial point, so
        // the mixed mode reports the fp64 solve's status there; the others leave at once
        bqp::OcpKernelArgs a3 = a;
        a3.hand_in = nullptr; a3.hand_it = nullptr; a3.redo_flag = hflag;
        a3.queue = nullptr;           // sparse: most workgroups leave at once
        HIP_TRY(bqp::launch_ocp(a3, nx, nu, np, st));
    } else if (f32) {
        HIP_TRY(bqp::launch_ocp_f32(a, nx, nu, np, st));
    } else {
        HIP_TRY(bqp::launch_ocp(a, nx, nu, np, st));
    }
    // repair launch (fp64): the instances the solve launch marked (0 / -8 exits; with polish 2
    // also weakly active rows) are solved again and polished to their active-set solution; a
    // workgroup with no marked instance leaves at once.  The mixed mode repairs with the
    // continuation's arguments.
    if (!f32 && a.polish > 0) HIP_TRY(bqp::launch_ocp(a, nx, nu, np, st, true));
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->timed = true;
    h->launches = (mixed ? 3 : 1) + ((!f32 && a.polish > 0) ? 1 : 0);
    if (out) HIP_TRY(bqp::launch_ocp_finalize(Sd, batch, out, st));
    return BQP_OK;
}

int bqp_solve_ocp_batched(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D,
                          const bqp_options* opt, double* x, double* u, double* theta,
                          double* fval, int* exitflag, bqp_output* out,
                          const bqp_ocp_duals* duals) {
    if (!h) return BQP_E_ARG;
    int rc = ocp_check(d, batch, D);
    if (rc) return rc;
    if (!x || !u || !theta || !exitflag) return BQP_E_ARG;
    DevScope ds(h->device);
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N, mp = d->n_poly;
    const size_t nv = nx + nu + np;
    // input spans (elements)
    struct In { const double* src; size_t n; double* dst; };
    In in[12] = {
        {D->A, span(batch, D->sA, nx * nx), nullptr},
        {D->B, span(batch, D->sB, nx * nu), nullptr},
        {D->c, D->c ? span(batch, D->sc, nx) : 0, nullptr},
        {D->W, span(batch, D->sW, (N + 1) * nv * nv), nullptr},
        {D->w, D->w ? span(batch, D->sw, (N + 1) * nv) : 0, nullptr},
        {D->xlb, D->xlb ? span(batch, D->sxb, (size_t)(N + 1) * nx) : 0, nullptr},
        {D->xub, D->xub ? span(batch, D->sxb, (size_t)(N + 1) * nx) : 0, nullptr},
        {D->ulb, D->ulb ? span(batch, D->sub, (size_t)N * nu) : 0, nullptr},
        {D->uub, D->uub ? span(batch, D->sub, (size_t)N * nu) : 0, nullptr},
        {D->Fp, mp > 0 ? span(batch, D->sFp, (size_t)mp * nv) : 0, nullptr},
        {D->hp, mp > 0 ? span(batch, D->shp, (size_t)mp) : 0, nullptr},
        {D->x0, span(batch, D->sx0, nx), nullptr},
    };
    const size_t nxo = (size_t)batch * (N + 1) * nx, nuo = (size_t)batch * N * nu,
                 nto = (size_t)batch * np, nfo = (size_t)batch;
    size_t ndual = 0;
    if (duals) ndual = (size_t)batch * ((size_t)N * nx + (size_t)(N + 1) * nx * 2 + (size_t)N * nu * 2 + mp);
    size_t total = 0;
    for (auto& e : in) total += e.n;
    total += nxo + nuo + nto + nfo + ndual;
    const size_t outbytes = sizeof(bqp_output) * (size_t)batch;
    const size_t bytes = sizeof(double) * (total + 16) + sizeof(int) * (size_t)batch + outbytes + 64;
    HIP_TRY(h->stage.reserve(bytes));
    double* cur = (double*)h->stage.p;
    for (auto& e : in) {
        if (e.n) {
            e.dst = cur;
            HIP_TRY(hipMemcpyAsync(cur, e.src, sizeof(double) * e.n, hipMemcpyHostToDevice, h->stream));
            cur += e.n;
        }
    }
    double* xd = cur; cur += nxo;
    double* ud = cur; cur += nuo;
    double* td = cur; cur += nto;
    double* fd = cur; cur += nfo;
    double* dual_base = cur; cur += ndual;
    int* ed = (int*)cur;
    bqp_output* od = (bqp_output*)(((uintptr_t)(ed + batch) + 63) & ~(uintptr_t)63);
    bqp_ocp_data Dd = *D;
    Dd.A = in[0].dst; Dd.B = in[1].dst; Dd.c = in[2].dst; Dd.W = in[3].dst; Dd.w = in[4].dst;
    Dd.xlb = in[5].dst; Dd.xub = in[6].dst; Dd.ulb = in[7].dst; Dd.uub = in[8].dst;
    Dd.Fp = in[9].dst; Dd.hp = in[10].dst; Dd.x0 = in[11].dst;
    bqp_ocp_duals dd;
    memset(&dd, 0, sizeof(dd));
    if (duals) {
        double* q = dual_base;
        dd.pi = q; q += (size_t)batch * N * nx;
        dd.lam_x = q; q += (size_t)batch * (N + 1) * nx * 2;
        dd.lam_u = q; q += (size_t)batch * N * nu * 2;
        dd.lam_p = q;
    }
    rc = bqp_solve_ocp_batched_device(h, d, batch, &Dd, opt, xd, ud, td, fd, ed,
                                      out ? od : nullptr, duals ? &dd : nullptr, h->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(x, xd, sizeof(double) * nxo, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(u, ud, sizeof(double) * nuo, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(theta, td, sizeof(double) * nto, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(exitflag, ed, sizeof(int) * batch, hipMemcpyDeviceToHost, h->stream));
    if (fval) HIP_TRY(hipMemcpyAsync(fval, fd, sizeof(double) * nfo, hipMemcpyDeviceToHost, h->stream));
    if (out) HIP_TRY(hipMemcpyAsync(out, od, outbytes, hipMemcpyDeviceToHost, h->stream));
    if (duals) {
        if (duals->pi) HIP_TRY(hipMemcpyAsync(duals->pi, dd.pi, sizeof(double) * batch * N * nx, hipMemcpyDeviceToHost, h->stream));
        if (duals->lam_x) HIP_TRY(hipMemcpyAsync(duals->lam_x, dd.lam_x, sizeof(double) * batch * (N + 1) * nx * 2, hipMemcpyDeviceToHost, h->stream));
        if (duals->lam_u) HIP_TRY(hipMemcpyAsync(duals->lam_u, dd.lam_u, sizeof(double) * batch * N * nu * 2, hipMemcpyDeviceToHost, h->stream));
        if (duals->lam_p && mp > 0) HIP_TRY(hipMemcpyAsync(duals->lam_p, dd.lam_p, sizeof(double) * batch * mp, hipMemcpyDeviceToHost, h->stream));
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

// ------------------------------------------------------------------------------------------
// dense quadprog
// ------------------------------------------------------------------------------------------
static int dense_check(const bqp_dims* d, int batch, const double* H, const double* f) {
    if (!d || batch <= 0 || !H || !f) return BQP_E_ARG;
    if (d->n <= 0 || d->m < 0 || d->me < 0) return BQP_E_ARG;
    if (d->n > 256 || d->me > 256 || d->m > 8192) return BQP_E_UNSUPPORTED;
    return BQP_OK;
}

int bqp_quadprog_batched_device(bqp_handle h, const bqp_dims* d, int batch, const bqp_strides* s,
                                const double* H, const double* f, const double* A,
                                const double* b, const double* Aeq, const double* beq,
                                const double* lb, const double* ub, const bqp_options* opt,
                                double* x, double* fval, int* exitflag, double* lam_ineqlin,
                                double* lam_eqlin, double* lam_lower, double* lam_upper,
                                bqp_output* out, void* stream) {
    if (!h) return BQP_E_ARG;
    int rc = dense_check(d, batch, H, f);
    if (rc) return rc;
    if (!x || !exitflag || !s) return BQP_E_ARG;
    if ((d->m > 0 && (!A || !b)) || (d->me > 0 && (!Aeq || !beq))) return BQP_E_ARG;
    DevScope ds(h->device);
    hipStream_t st = (hipStream_t)stream;
    bqp_options o;
    resolve(opt, &o);
    const int64_t wst = bqp::dense_work_doubles(d->n, d->m, d->me);
    HIP_TRY(h->dwork.reserve(sizeof(double) * ((size_t)wst * batch + (size_t)batch * bqp::STATS_W + 8)));
    double* wk = (double*)h->dwork.p;
    double* Sd = wk + (size_t)wst * batch;
    bqp::DenseKernelArgs a;
    memset(&a, 0, sizeof(a));
    a.n = d->n; a.m = d->m; a.me = d->me; a.batch = batch; a.max_iter = o.max_iter;
    a.tol_stat = o.tol_stat; a.tol_feas = o.tol_feas; a.tol_comp = o.tol_comp; a.tau = o.tau;
    a.H = H; a.f = f; a.A = A; a.b = b; a.Aeq = Aeq; a.beq = beq; a.lb = lb; a.ub = ub;
    a.sH = s->sH; a.sf = s->sf; a.sA = s->sA; a.sb = s->sb; a.sAeq = s->sAeq; a.sbeq = s->sbeq;
    a.slb = s->slb; a.sub = s->sub;
    a.x = x; a.fval = fval; a.lam_ineqlin = lam_ineqlin; a.lam_eqlin = lam_eqlin;
    a.lam_lower = lam_lower; a.lam_upper = lam_upper; a.exitflag = exitflag; a.stats = Sd;
    a.work = wk; a.work_stride = wst;
    a.polish = o.polish < 0 ? 0 : 1;
    HIP_TRY(hipEventRecord(h->ev0, st));
    HIP_TRY(bqp::launch_dense(a, st));
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->timed = true;
    h->launches = 1;
    if (out) HIP_TRY(bqp::launch_ocp_finalize(Sd, batch, out, st));
    return BQP_OK;
}

int bqp_quadprog_batched(bqp_handle h, const bqp_dims* d, int batch, const bqp_strides* s,
                         const double* H, const double* f, const double* A, const double* b,
                         const double* Aeq, const double* beq, const double* lb, const double* ub,
                         const double* x0, const bqp_options* opt, double* x, double* fval,
                         int* exitflag, double* lam_ineqlin, double* lam_eqlin,
                         double* lam_lower, double* lam_upper, bqp_output* out) {
    (void)x0;
    if (!h) return BQP_E_ARG;
    int rc = dense_check(d, batch, H, f);
    if (rc) return rc;
    if (!x || !exitflag) return BQP_E_ARG;
    bqp_strides zs;
    memset(&zs, 0, sizeof(zs));
    if (!s) s = &zs;
    DevScope ds(h->device);
    const size_t n = d->n, m = d->m, me = d->me;
    struct In { const double* src; size_t n; double* dst; };
    In in[8] = {
        {H, span(batch, s->sH, n * n), nullptr},
        {f, span(batch, s->sf, n), nullptr},
        {A, (A && m) ? span(batch, s->sA, m * n) : 0, nullptr},
        {b, (b && m) ? span(batch, s->sb, m) : 0, nullptr},
        {Aeq, (Aeq && me) ? span(batch, s->sAeq, me * n) : 0, nullptr},
        {beq, (beq && me) ? span(batch, s->sbeq, me) : 0, nullptr},
        {lb, lb ? span(batch, s->slb, n) : 0, nullptr},
        {ub, ub ? span(batch, s->sub, n) : 0, nullptr},
    };
    size_t total = 0;
    for (auto& e : in) total += e.n;
    const size_t nxo = (size_t)batch * n, nli = (size_t)batch * m, nle = (size_t)batch * me;
    total += nxo + batch + nli + nle + 2 * nxo;
    const size_t outbytes = sizeof(bqp_output) * (size_t)batch;
    HIP_TRY(h->stage.reserve(sizeof(double) * (total + 16) + sizeof(int) * batch + outbytes + 64));
    double* cur = (double*)h->stage.p;
    for (auto& e : in)
        if (e.n) {
            e.dst = cur;
            HIP_TRY(hipMemcpyAsync(cur, e.src, sizeof(double) * e.n, hipMemcpyHostToDevice, h->stream));
            cur += e.n;
        }
    // quadprog semantics: the symmetric part of H (a no-op on a symmetric H)
    HIP_TRY(bqp::launch_dense_symmetrize(in[0].dst, (int)n, s->sH ? batch : 1, s->sH, h->stream));
    double* xd = cur; cur += nxo;
    double* fd = cur; cur += batch;
    double* lid = cur; cur += nli;
    double* led = cur; cur += nle;
    double* lld = cur; cur += nxo;
    double* lud = cur; cur += nxo;
    int* ed = (int*)cur;
    bqp_output* od = (bqp_output*)(((uintptr_t)(ed + batch) + 63) & ~(uintptr_t)63);
    rc = bqp_quadprog_batched_device(h, d, batch, s, in[0].dst, in[1].dst, in[2].dst, in[3].dst,
                                     in[4].dst, in[5].dst, in[6].dst, in[7].dst, opt, xd, fd, ed,
                                     lid, led, lld, lud, out ? od : nullptr, h->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(x, xd, sizeof(double) * nxo, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(exitflag, ed, sizeof(int) * batch, hipMemcpyDeviceToHost, h->stream));
    if (fval) HIP_TRY(hipMemcpyAsync(fval, fd, sizeof(double) * batch, hipMemcpyDeviceToHost, h->stream));
    if (lam_ineqlin && m) HIP_TRY(hipMemcpyAsync(lam_ineqlin, lid, sizeof(double) * nli, hipMemcpyDeviceToHost, h->stream));
    if (lam_eqlin && me) HIP_TRY(hipMemcpyAsync(lam_eqlin, led, sizeof(double) * nle, hipMemcpyDeviceToHost, h->stream));
    if (lam_lower) HIP_TRY(hipMemcpyAsync(lam_lower, lld, sizeof(double) * nxo, hipMemcpyDeviceToHost, h->stream));
    if (lam_upper) HIP_TRY(hipMemcpyAsync(lam_upper, lud, sizeof(double) * nxo, hipMemcpyDeviceToHost, h->stream));
    if (out) HIP_TRY(hipMemcpyAsync(out, od, outbytes, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

// ------------------------------------------------------------------------------------------
// learning-based MPC: Nadaraya-Watson oracle and the Gauss-Newton SQP (bqp_lbmpc.hip)
// ------------------------------------------------------------------------------------------
#define LB_NTRIAL 8
// SQP iterations at one step after which every QP sub-problem is polished (bqp_lbmpc_solve_batched)
constexpr int LB_POLISH_STALL = 6;

int bqp_nw_oracle_device(bqp_handle h, int batch, int q, const double* data, int64_t sdata,
                         const double* xi, double* g, double* dg, double bandwidth,
                         double lambda, void* stream) {
    if (!h || batch <= 0 || q <= 0 || !data || !xi || !g) return BQP_E_ARG;
    if (q > 512) return BQP_E_UNSUPPORTED;
    DevScope ds(h->device);
    const double bw = bandwidth > 0 ? bandwidth : 0.5, lam = lambda > 0 ? lambda : 1e-3;
    HIP_TRY(bqp::launch_nw_oracle(batch, q, data, sdata, xi, g, dg, bw, lam, (hipStream_t)stream));
    return BQP_OK;
}

int bqp_nw_oracle(bqp_handle h, int batch, int q, const double* data, int64_t sdata,
                  const double* xi, double* g, double* dg, double bandwidth, double lambda) {
    if (!h || batch <= 0 || q <= 0 || !data || !xi || !g) return BQP_E_ARG;
    if (q > 512) return BQP_E_UNSUPPORTED;
    DevScope ds(h->device);
    const size_t nd = span(batch, sdata, (size_t)7 * q);
    const size_t tot = nd + (3 + 4 + 12) * (size_t)batch;
    HIP_TRY(h->stage.reserve(sizeof(double) * tot));
    double* dd = (double*)h->stage.p;
    double* dx = dd + nd;
    double* dgv = dx + 3 * (size_t)batch;
    double* ddg = dgv + 4 * (size_t)batch;
    HIP_TRY(hipMemcpyAsync(dd, data, sizeof(double) * nd, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipMemcpyAsync(dx, xi, sizeof(double) * 3 * batch, hipMemcpyHostToDevice, h->stream));
    int rc = bqp_nw_oracle_device(h, batch, q, dd, sdata, dx, dgv, ddg, bandwidth, lambda, h->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(g, dgv, sizeof(double) * 4 * batch, hipMemcpyDeviceToHost, h->stream));
    if (dg) HIP_TRY(hipMemcpyAsync(dg, ddg, sizeof(double) * 12 * batch, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

static int lbmpc_check(const bqp_lbmpc_dims* d, int batch, const bqp_lbmpc_data* D) {
    if (!d || !D || batch <= 0) return BQP_E_ARG;
    if (d->N <= 0 || d->n_run < 0 || d->n_run > d->N || d->q <= 0 || d->m < 0 ||
        (d->mask != 0 && d->mask != 1) || (d->hessian != 0 && d->hessian != 1))
        return BQP_E_ARG;
    if (!D->A || !D->B || !D->K || !D->Lq || !D->Lr || !D->Lp || !D->Lt || !D->LAMBDA ||
        !D->PSI || !D->xs || !D->data || !D->x0 || (d->m > 0 && (!D->Ain || !D->bin)))
        return BQP_E_ARG;
    const int n = d->N * d->nu + d->np;
    if (!bqp::lbmpc_supported(d->nx, d->nu, d->np, n, d->q) || d->m > 8192) return BQP_E_UNSUPPORTED;
    return BQP_OK;
}

// the learned-model SQP's kernel arguments and per-instance state (done, iteration counts, flags
// zeroed), and the QP sub-problem's dense-kernel arguments: shared by the batched solve and the
// asynchronous closed loop
static hipError_t lbmpc_setup(bqp_handle h, const bqp_lbmpc_dims* d, int batch, const bqp_lbmpc_data* D,
                              const bqp_options& o, double* z, double* lam, int* exitflag, int* iterations,
                              hipStream_t st, bqp::LbmpcArgs& a, bqp::DenseKernelArgs& q) {
    const int N = d->N, n = N * d->nu + d->np, m = d->m;
    const int nr = d->n_run * (d->nx + d->nu) + 2 * d->nx;
    const size_t B = batch;
    const size_t n2 = d->hessian ? B * 3 * (size_t)N * n : 0;   // Jr2, Tr2 of the exact Hessian
    const size_t nd = B * nr * n + B * nr + B * n * n + B * n + 2 * B * m + B * n + B +
                      B * LB_NTRIAL + 2 * B + 2 * n2;
    const size_t ni = 3 * B + 4;
    hipError_t e = h->lwork.reserve(sizeof(double) * nd + sizeof(int) * ni);
    if (e != hipSuccess) return e;
    double* p = (double*)h->lwork.p;
    memset(&a, 0, sizeof(a));
    a.Jr = p; p += B * nr * n;
    a.er = p; p += B * nr;
    a.H = p; p += B * n * n;
    a.f = p; p += B * n;
    a.bsh = p; p += B * m;
    double* lam_int = p; p += B * m;
    a.d = p; p += B * n;
    a.cost0 = p; p += B;
    a.costT = p; p += B * LB_NTRIAL;
    a.stat = p; p += B;
    a.cprev = p; p += B;
    a.Jr2 = p; p += n2;
    a.Tr2 = p; p += n2;
    int* ip = (int*)p;
    a.qpflag = ip; ip += B;
    a.hused = ip; ip += B;
    a.done = ip; ip += B;
    a.ndone = ip;
    // exact Hessian where its LDS fits (n <= 127), Gauss-Newton otherwise (include/bqp.h)
    a.hess = d->hessian && bqp::lbmpc_hess_fits(n);
    a.lam = lam ? lam : lam_int;
    a.z = z; a.flag = exitflag; a.iters = iterations;
    a.N = N; a.n = n; a.nr = nr; a.m = m; a.q = d->q; a.n_run = d->n_run;
    a.term_learned = d->term_learned; a.batch = batch; a.ntrial = LB_NTRIAL;
    a.wrows = d->mask ? 8 : 7;
    a.max_iter = o.max_iter;
    const double bw = D->bandwidth > 0 ? D->bandwidth : 0.5;
    a.hinv2 = 1.0 / (bw * bw);
    a.lam_nw = D->lambda > 0 ? D->lambda : 1e-3;
    a.tol_step = o.tol_stat;            // |d| <= tol_stat (1 + |z|)
    a.tol_stat = 10.0 * o.tol_stat;     // |grad J + Ain' lam| <= 10 tol_stat (1 + |grad J|)
    a.A = D->A; a.B = D->B; a.K = D->K; a.Lq = D->Lq; a.Lr = D->Lr; a.Lp = D->Lp; a.Lt = D->Lt;
    a.LAM = D->LAMBDA; a.PSI = D->PSI; a.xs = D->xs;
    a.data = D->data; a.sdata = D->sdata; a.x0 = D->x0; a.sx0 = D->sx0;
    a.Ain = D->Ain; a.bin = D->bin; a.sbin = D->sbin;
    if ((e = hipMemsetAsync(a.done, 0, sizeof(int) * (B + 1), st)) != hipSuccess) return e;   // done[], ndone
    if ((e = hipMemsetAsync(a.hused, 0, sizeof(int) * B, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.iters, 0, sizeof(int) * B, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.flag, 0, sizeof(int) * B, st)) != hipSuccess) return e;
    // QP sub-problem (dense kernel): min 0.5 d'Hd + f'd  s.t.  Ain d <= bin - Ain z
    const int64_t wst = bqp::dense_work_doubles(n, m, 0);
    if ((e = h->dwork.reserve(sizeof(double) * ((size_t)wst * B + B * bqp::STATS_W + 8))) != hipSuccess) return e;
    memset(&q, 0, sizeof(q));
    q.n = n; q.m = m; q.me = 0; q.batch = batch; q.max_iter = 100;
    q.tol_stat = 1e-8; q.tol_feas = 1e-10; q.tol_comp = 1e-14; q.tau = 0.995;   // bqp_default_options
    q.H = a.H; q.f = a.f; q.A = D->Ain; q.b = a.bsh;
    q.sH = (int64_t)n * n; q.sf = n; q.sA = 0; q.sb = m;
    q.x = a.d; q.lam_ineqlin = a.lam; q.exitflag = a.qpflag;
    q.work = (double*)h->dwork.p; q.work_stride = wst;
    // sub-problem polish after 0 / -8 exits (modes 0-2; mode 3: not before the stall), and on every
    // sub-problem (mode 2) once the SQP has run LB_POLISH_STALL iterations at a step: the Gauss-Newton iteration converges linearly on the learned costs of
    // DMS_LBMPC_casadi.m and interior-point steps accurate to ~1e-8 left it wandering at that level
    // (tools/diag_dms_gpu.py); with the exact Hessian the SQP ends in 1-4 iterations.  Before the
    // stall, mode 3 (the closed loop's default) leaves -8 exits unpolished: in the learned loop ~10 %
    // of the sub-problems end -8 once mu ~ 1e-15 (the factor leaves fp64 range one step past an
    // accurate iterate, which the update kernel takes as is), and the polish launch for them was
    // ~1/3 of each SQP iteration (5.5 of 16 ms, BQP_LB_TRACE=2).  A single solve keeps mode 1: its
    // weakly determined tail inputs move ~1e-6 without the polish.
    // instances whose SQP has finished are not solved again (the update kernel skips them too)
    q.skip = a.done;
    q.stats = (double*)h->dwork.p + (size_t)wst * B;
    return hipSuccess;
}

int bqp_lbmpc_solve_batched_device(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                                   const bqp_lbmpc_data* D, const bqp_options* opt, double* z,
                                   double* lam, double* cost, int* exitflag, int* iterations,
                                   void* stream) {
    if (!h) return BQP_E_ARG;
    int rc = lbmpc_check(d, batch, D);
    if (rc) return rc;
    if (!z || !exitflag || !iterations) return BQP_E_ARG;
    DevScope ds(h->device);
    hipStream_t st = (hipStream_t)stream;
    bqp_options o;
    resolve(opt, &o);
    const int N = d->N, n = N * d->nu + d->np;
    const size_t B = batch;
    bqp::LbmpcArgs a;
    bqp::DenseKernelArgs q;
    HIP_TRY(lbmpc_setup(h, d, batch, D, o, z, lam, exitflag, iterations, st, a, q));
    (void)n;
    HIP_TRY(hipEventRecord(h->ev0, st));
    int launches = 0;
    // diagnostic (BQP_LB_TRACE=2): per-launch event times of the first SQP iterations
    const char* lbt = getenv("BQP_LB_TRACE");
    const bool lbt2 = lbt && atoi(lbt) >= 2;
    EventGuard tg[6];                      // released on every return path
    hipEvent_t tev[6] = {};
    if (lbt2)
        for (int k = 0; k < 6; ++k) { HIP_TRY(hipEventCreate(&tg[k].e)); tev[k] = tg[k].e; }
    for (int it = 0; it < o.max_iter; ++it) {
        if (lbt2) HIP_TRY(hipEventRecord(tev[0], st));
        HIP_TRY(bqp::launch_lbmpc_rollout(a, 1, st));
        if (lbt2) HIP_TRY(hipEventRecord(tev[1], st));
        HIP_TRY(bqp::launch_lbmpc_normal(a, st));
        if (a.hess) HIP_TRY(bqp::launch_lbmpc_hess(a, st));
        if (lbt2) HIP_TRY(hipEventRecord(tev[2], st));
        q.polish = o.polish < 0 ? 0 : (it >= LB_POLISH_STALL ? 2 : (o.polish == 3 ? 0 : 1));
        HIP_TRY(bqp::launch_dense(q, st));
        if (lbt2) {
            HIP_TRY(hipEventRecord(tev[3], st));
            HIP_TRY(bqp::launch_lbmpc_rollout(a, 0, st));
            HIP_TRY(hipEventRecord(tev[4], st));
            HIP_TRY(bqp::launch_lbmpc_update(a, st));
            HIP_TRY(hipEventRecord(tev[5], st));
            HIP_TRY(hipEventSynchronize(tev[5]));
            float ms[5];
            for (int k = 0; k < 5; ++k) HIP_TRY(hipEventElapsedTime(&ms[k], tev[k], tev[k + 1]));
            fprintf(stderr, "bqp sqp it %d ms: rollout+sens %.3f normal+hess %.3f dense(+polish) %.3f trials %.3f update %.3f\n",
                    it, ms[0], ms[1], ms[2], ms[3], ms[4]);
        }
        if (lbt && !lbt2) {     // diagnostic: sub-problem exit flags per SQP iteration
            std::vector<int> fl(batch), dn(batch);
            HIP_TRY(hipMemcpyAsync(fl.data(), a.qpflag, sizeof(int) * batch, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(dn.data(), a.done, sizeof(int) * batch, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            int c1 = 0, c0 = 0, c8 = 0, co = 0, act = 0;
            for (int b = 0; b < batch; ++b) {
                if (dn[b]) continue;
                ++act;
                if (fl[b] == 1) ++c1; else if (fl[b] == 0) ++c0; else if (fl[b] == -8) ++c8; else ++co;
            }
            fprintf(stderr, "bqp sqp it %d: active %d, sub-problem flags 1:%d 0:%d -8:%d other:%d\n", it, act,
                    c1, c0, c8, co);
        }
        if (!lbt2) {
            HIP_TRY(bqp::launch_lbmpc_rollout(a, 0, st));
            HIP_TRY(bqp::launch_lbmpc_update(a, st));
        }
        launches += a.hess ? 6 : 5;
        // the batch is done when every instance is: polled after each iteration for large
        // sub-problems (an SQP iteration is ~20 ms of kernels at the learned loop's N = 100 shape,
        // and polling every 4th ran up to three iterations past the last instance's convergence),
        // every 4th for small ones (the host round trip against ~0.3 ms iterations at N = 10)
        if ((it + 1) % (n >= 64 ? 1 : 4) == 0 || it + 1 == o.max_iter) {
            int nd_h = 0;
            HIP_TRY(hipMemcpyAsync(&nd_h, a.ndone, sizeof(int), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (nd_h >= batch) break;
        }
    }
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->timed = true;
    h->launches = launches;
    if (cost) HIP_TRY(hipMemcpyAsync(cost, a.cost0, sizeof(double) * B, hipMemcpyDeviceToDevice, st));
    return BQP_OK;
}

int bqp_lbmpc_solve_batched(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                            const bqp_lbmpc_data* D, const bqp_options* opt, double* z,
                            double* lam, double* cost, int* exitflag, int* iterations) {
    if (!h) return BQP_E_ARG;
    int rc = lbmpc_check(d, batch, D);
    if (rc) return rc;
    if (!z || !exitflag || !iterations) return BQP_E_ARG;
    DevScope ds(h->device);
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N, m = d->m;
    const int n = N * nu + np;
    struct In { const double* src; size_t n; double* dst; };
    In in[] = {
        {D->A, (size_t)nx * nx, nullptr}, {D->B, (size_t)nx * nu, nullptr},
        {D->K, (size_t)nu * nx, nullptr}, {D->Lq, (size_t)nx * nx, nullptr},
        {D->Lr, (size_t)nu * nu, nullptr}, {D->Lp, (size_t)nx * nx, nullptr},
        {D->Lt, (size_t)nx * nx, nullptr}, {D->LAMBDA, (size_t)nx * np, nullptr},
        {D->PSI, (size_t)nu * np, nullptr}, {D->xs, (size_t)nx, nullptr},
        {D->data, span(batch, D->sdata, (size_t)(d->mask ? 8 : 7) * d->q), nullptr},
        {D->x0, span(batch, D->sx0, nx), nullptr},
        {D->Ain, (size_t)m * n, nullptr}, {D->bin, span(batch, D->sbin, m), nullptr},
        {z, (size_t)batch * n, nullptr},
    };
    const int nin = sizeof(in) / sizeof(in[0]);
    size_t tot = 0;
    for (int i = 0; i < nin; ++i) tot += (in[i].src ? in[i].n : 0);
    const size_t nlam = (size_t)batch * m;
    tot += nlam + batch;
    HIP_TRY(h->stage.reserve(sizeof(double) * tot + sizeof(int) * 2 * (size_t)batch));
    double* cur = (double*)h->stage.p;
    for (int i = 0; i < nin; ++i) {
        if (!in[i].src || in[i].n == 0) continue;
        in[i].dst = cur;
        HIP_TRY(hipMemcpyAsync(cur, in[i].src, sizeof(double) * in[i].n, hipMemcpyHostToDevice, h->stream));
        cur += in[i].n;
    }
    double* zd = in[nin - 1].dst;
    double* ld = cur; cur += nlam;
    double* cd = cur; cur += batch;
    int* ed = (int*)cur;
    int* itd = ed + batch;
    bqp_lbmpc_data Dd = *D;
    Dd.A = in[0].dst; Dd.B = in[1].dst; Dd.K = in[2].dst; Dd.Lq = in[3].dst; Dd.Lr = in[4].dst;
    Dd.Lp = in[5].dst; Dd.Lt = in[6].dst; Dd.LAMBDA = in[7].dst; Dd.PSI = in[8].dst;
    Dd.xs = in[9].dst; Dd.data = in[10].dst; Dd.x0 = in[11].dst; Dd.Ain = in[12].dst;
    Dd.bin = in[13].dst;
    rc = bqp_lbmpc_solve_batched_device(h, d, batch, &Dd, opt, zd, ld, cd, ed, itd, h->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(z, zd, sizeof(double) * batch * n, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(exitflag, ed, sizeof(int) * batch, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(iterations, itd, sizeof(int) * batch, hipMemcpyDeviceToHost, h->stream));
    if (lam && m) HIP_TRY(hipMemcpyAsync(lam, ld, sizeof(double) * nlam, hipMemcpyDeviceToHost, h->stream));
    if (cost) HIP_TRY(hipMemcpyAsync(cost, cd, sizeof(double) * batch, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

// ------------------------------------------------------------------------------------------
// closed-loop simulation: batched structured solve + true-plant step, per time step
// ------------------------------------------------------------------------------------------
static int closed_loop_impl(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D,
                            const bqp_options* opt, const bqp_closed_loop* cl,
                            const bqp_learning* lw, const double* x_init, double* X, double* U,
                            int* exitflag, void* stream) {
    if (!h || !cl || !x_init || !X || !U) return BQP_E_ARG;
    int rc = ocp_check(d, batch, D);
    if (rc) return rc;
    if ((cl->plant != BQP_PLANT_MG_RK4 && cl->plant != BQP_PLANT_MG_ODE23) || cl->steps <= 0 || !(cl->delta > 0) || !cl->x_eq || !cl->u_eq)
        return BQP_E_ARG;
    if (d->nx != 4 || d->nu != 1) return BQP_E_UNSUPPORTED;   // the MG plant
    if (lw && (lw->q < 1 || lw->q > (1 << 20) || !lw->XL)) return BQP_E_ARG;
    DevScope ds(h->device);
    hipStream_t st = (hipStream_t)stream;
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N;
    const size_t B = batch;
    const size_t nwin = lw ? B * (size_t)lw->q * 8 : 0;
    const size_t nd = B * nx + B * (N + 1) * nx + B * N * nu + B * np + nwin;
    HIP_TRY(h->cwork.reserve(sizeof(double) * nd + sizeof(int) * B));
    double* s = (double*)h->cwork.p;
    double* xo = s + B * nx;
    double* uo = xo + B * (N + 1) * nx;
    double* th = uo + B * N * nu;
    double* win = th + B * np;
    int* fl = (int*)(win + nwin);
    if (lw && lw->window) win = lw->window;   // the caller's buffer (device) keeps the final window
    HIP_TRY(bqp::launch_closed_loop_init(batch, nx, cl->steps, x_init, cl->x_eq, s, X, st));
    const double bw = (lw && lw->bandwidth > 0) ? lw->bandwidth : 0.5;
    const double lam = (lw && lw->lambda > 0) ? lw->lambda : 1e-3;
    if (lw) HIP_TRY(bqp::launch_lbmpc_window_init(batch, cl->steps, lw->q, lw->mask, x_init, win, lw->XL, st));
    bqp_ocp_data Dm = *D;
    Dm.x0 = s;
    Dm.sx0 = nx;
    EventGuard e0;
    HIP_TRY(hipEventCreate(&e0.e));
    HIP_TRY(hipEventRecord(e0.e, st));
    int launches = 0;
    for (int t = 0; t < cl->steps; ++t) {
        rc = bqp_solve_ocp_batched_device(h, d, batch, &Dm, opt, xo, uo, th, nullptr, fl, nullptr,
                                          nullptr, stream);
        if (rc) return rc;
        launches += h->launches + (lw ? 2 : 1);
        HIP_TRY(bqp::launch_mg_plant(cl->plant, batch, N, cl->steps, t, cl->delta, uo, fl, cl->x_eq, cl->u_eq,
                                     s, X, U, exitflag, st));
        if (lw)
            HIP_TRY(bqp::launch_lbmpc_window(batch, cl->steps, t, lw->q, bw, lam, D->A, D->sA, D->B,
                                             D->sB, cl->x_eq, cl->u_eq, X, U, win, lw->XL, st));
    }
    // timing of the whole loop (solves + plant steps) on this stream
    HIP_TRY(hipEventRecord(h->ev1, st));
    HIP_TRY(hipEventSynchronize(h->ev1));
    std::swap(h->ev0, e0.e);   // the guard destroys the previous start event
    h->timed = true;
    h->launches = launches;
    return BQP_OK;
}

int bqp_closed_loop_ocp_device(bqp_handle h, const bqp_ocp_dims* d, int batch,
                               const bqp_ocp_data* D, const bqp_options* opt,
                               const bqp_closed_loop* cl, const double* x_init, double* X,
                               double* U, int* exitflag, void* stream) {
    return closed_loop_impl(h, d, batch, D, opt, cl, nullptr, x_init, X, U, exitflag, stream);
}

int bqp_closed_loop_lbmpc_device(bqp_handle h, const bqp_ocp_dims* d, int batch,
                                 const bqp_ocp_data* D, const bqp_options* opt,
                                 const bqp_closed_loop* cl, const bqp_learning* lw,
                                 const double* x_init, double* X, double* U, int* exitflag,
                                 void* stream) {
    if (!lw) return BQP_E_ARG;
    return closed_loop_impl(h, d, batch, D, opt, cl, lw, x_init, X, U, exitflag, stream);
}

static int closed_loop_host(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D,
                            const bqp_options* opt, const bqp_closed_loop* cl,
                            const bqp_learning* lw, const double* x_init, double* X, double* U,
                            int* exitflag) {
    if (!h || !cl || !x_init || !X || !U) return BQP_E_ARG;
    if (lw && (lw->q < 1 || lw->q > (1 << 20) || !lw->XL)) return BQP_E_ARG;
    int rc = ocp_check(d, batch, D);
    if (rc) return rc;
    // validate the loop description before sizing the staging buffers from it
    if ((cl->plant != BQP_PLANT_MG_RK4 && cl->plant != BQP_PLANT_MG_ODE23) || cl->steps <= 0 || !(cl->delta > 0) || !cl->x_eq || !cl->u_eq)
        return BQP_E_ARG;
    if (d->nx != 4 || d->nu != 1) return BQP_E_UNSUPPORTED;
    DevScope ds(h->device);
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N, mp = d->n_poly;
    const int nv = nx + nu + np;
    struct In { const double* src; size_t n; double* dst; };
    In in[] = {
        {D->A, span(batch, D->sA, (size_t)nx * nx), nullptr},
        {D->B, span(batch, D->sB, (size_t)nx * nu), nullptr},
        {D->c, D->c ? span(batch, D->sc, nx) : 0, nullptr},
        {D->W, span(batch, D->sW, (size_t)(N + 1) * nv * nv), nullptr},
        {D->w, D->w ? span(batch, D->sw, (size_t)(N + 1) * nv) : 0, nullptr},
        {D->xlb, D->xlb ? span(batch, D->sxb, (size_t)(N + 1) * nx) : 0, nullptr},
        {D->xub, D->xub ? span(batch, D->sxb, (size_t)(N + 1) * nx) : 0, nullptr},
        {D->ulb, D->ulb ? span(batch, D->sub, (size_t)N * nu) : 0, nullptr},
        {D->uub, D->uub ? span(batch, D->sub, (size_t)N * nu) : 0, nullptr},
        {D->Fp, mp > 0 ? span(batch, D->sFp, (size_t)mp * nv) : 0, nullptr},
        {D->hp, mp > 0 ? span(batch, D->shp, mp) : 0, nullptr},
        {x_init, (size_t)batch * nx, nullptr},
        {cl->x_eq, (size_t)nx, nullptr},
        {cl->u_eq, (size_t)nu, nullptr},
    };
    const int nin = sizeof(in) / sizeof(in[0]);
    const size_t nX = (size_t)batch * (cl->steps + 1) * nx, nU = (size_t)batch * cl->steps * nu;
    const size_t nW = lw ? (size_t)batch * lw->q * 8 : 0;
    size_t tot = nX + nU + (lw ? nX + nW : 0);
    for (int i = 0; i < nin; ++i) tot += (in[i].src ? in[i].n : 0);
    HIP_TRY(h->stage.reserve(sizeof(double) * tot + sizeof(int) * (size_t)batch * cl->steps));
    double* cur = (double*)h->stage.p;
    for (int i = 0; i < nin; ++i) {
        if (!in[i].src || in[i].n == 0) continue;
        in[i].dst = cur;
        HIP_TRY(hipMemcpyAsync(cur, in[i].src, sizeof(double) * in[i].n, hipMemcpyHostToDevice, h->stream));
        cur += in[i].n;
    }
    double* Xd = cur; cur += nX;
    double* Ud = cur; cur += nU;
    double* XLd = nullptr;
    double* Wd = nullptr;
    if (lw) { XLd = cur; cur += nX; Wd = cur; cur += nW; }
    int* Fd = (int*)cur;
    bqp_ocp_data Dd = *D;
    Dd.A = in[0].dst; Dd.B = in[1].dst; Dd.c = in[2].dst; Dd.W = in[3].dst; Dd.w = in[4].dst;
    Dd.xlb = in[5].dst; Dd.xub = in[6].dst; Dd.ulb = in[7].dst; Dd.uub = in[8].dst;
    Dd.Fp = in[9].dst; Dd.hp = in[10].dst;
    Dd.x0 = in[11].dst;   // placeholder (the loop feeds the measured states)
    bqp_closed_loop cd = *cl;
    cd.x_eq = in[12].dst; cd.u_eq = in[13].dst;
    bqp_learning ld;
    if (lw) { ld = *lw; ld.XL = XLd; ld.window = Wd; }
    rc = closed_loop_impl(h, d, batch, &Dd, opt, &cd, lw ? &ld : nullptr, in[11].dst, Xd, Ud,
                          exitflag ? Fd : nullptr, h->stream);
    if (rc) return rc;
    if (lw) {
        HIP_TRY(hipMemcpyAsync(lw->XL, XLd, sizeof(double) * nX, hipMemcpyDeviceToHost, h->stream));
        if (lw->window) HIP_TRY(hipMemcpyAsync(lw->window, Wd, sizeof(double) * nW, hipMemcpyDeviceToHost, h->stream));
    }
    HIP_TRY(hipMemcpyAsync(X, Xd, sizeof(double) * nX, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(U, Ud, sizeof(double) * nU, hipMemcpyDeviceToHost, h->stream));
    if (exitflag) HIP_TRY(hipMemcpyAsync(exitflag, Fd, sizeof(int) * (size_t)batch * cl->steps, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

int bqp_closed_loop_ocp(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D,
                        const bqp_options* opt, const bqp_closed_loop* cl, const double* x_init,
                        double* X, double* U, int* exitflag) {
    return closed_loop_host(h, d, batch, D, opt, cl, nullptr, x_init, X, U, exitflag);
}

int bqp_closed_loop_lbmpc(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D,
                          const bqp_options* opt, const bqp_closed_loop* cl,
                          const bqp_learning* lw, const double* x_init, double* X, double* U,
                          int* exitflag) {
    if (!lw) return BQP_E_ARG;
    return closed_loop_host(h, d, batch, D, opt, cl, lw, x_init, X, U, exitflag);
}

// ------------------------------------------------------------------------------------------
// learned-model NLP closed loop: batched SQP + true-plant step + data window, per time step
// ------------------------------------------------------------------------------------------
static int sqp_loop_check(const bqp_lbmpc_dims* d, int batch, const bqp_lbmpc_data* D,
                          const bqp_sqp_loop* sl, const bqp_closed_loop* cl,
                          const bqp_learning* lw, const double* x_init, const double* X,
                          const double* U) {
    if (!d || !D || !sl || !cl || !lw || !x_init || !X || !U || batch <= 0) return BQP_E_ARG;
    if ((cl->plant != BQP_PLANT_MG_RK4 && cl->plant != BQP_PLANT_MG_ODE23) || cl->steps <= 0 || !(cl->delta > 0) || !cl->x_eq || !cl->u_eq)
        return BQP_E_ARG;
    if (d->nx != 4 || d->nu != 1) return BQP_E_UNSUPPORTED;   // the MG plant
    if (lw->q != d->q || !lw->XL || (lw->mask != 0 && lw->mask != 1)) return BQP_E_ARG;
    if (d->m > 0 && (!sl->bin0 || !sl->Bx)) return BQP_E_ARG;
    // the loop supplies the window, the measured state and the rhs: check the rest
    bqp_lbmpc_data Dc = *D;
    double dummy = 0.0;
    Dc.data = &dummy; Dc.x0 = &dummy; Dc.bin = &dummy;
    bqp_lbmpc_dims dc = *d;
    dc.mask = 1;
    return lbmpc_check(&dc, batch, &Dc);
}

int bqp_closed_loop_sqp_device(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                               const bqp_lbmpc_data* D, const bqp_sqp_loop* sl,
                               const bqp_options* opt, const bqp_closed_loop* cl,
                               const bqp_learning* lw, const double* x_init, double* X, double* U,
                               int* exitflag, void* stream) {
    if (!h) return BQP_E_ARG;
    int rc = sqp_loop_check(d, batch, D, sl, cl, lw, x_init, X, U);
    if (rc) return rc;
    DevScope ds(h->device);
    hipStream_t st = (hipStream_t)stream;
    const int nx = d->nx, N = d->N, m = d->m, q = d->q;
    const int n = N * d->nu + d->np;
    const size_t B = batch;
    const size_t nd = B * nx + B * n + B * m + B + B * (size_t)q * 8;
    HIP_TRY(h->cwork.reserve(sizeof(double) * nd + sizeof(int) * (3 * B + 2)));
    double* s = (double*)h->cwork.p;     // measured deviation state
    double* z = s + B * nx;               // SQP iterate / solution
    double* bin = z + B * n;              // rhs of the step's constraints
    double* uo = bin + B * m;             // first input (deviation)
    double* win = uo + B;                 // window ring, 8 doubles per point
    int* fl = (int*)(win + B * (size_t)q * 8);
    int* it = fl + B;
    if (lw->window) win = lw->window;
    bqp_options ol;                       // the loop's default polish: only once the SQP stalls
    resolve(opt, &ol);
    if (ol.polish == 0) ol.polish = 3;
    opt = &ol;
    HIP_TRY(bqp::launch_closed_loop_init(batch, nx, cl->steps, x_init, cl->x_eq, s, X, st));
    HIP_TRY(bqp::launch_lbmpc_window_init(batch, cl->steps, q, lw->mask, x_init, win, lw->XL, st));
    HIP_TRY(hipMemsetAsync(z, 0, sizeof(double) * B * n, st));
    // the learned model's NW parameters: the loop's (bqp_learning) when set, else the model's own
    // (bqp_lbmpc_data, oracleL2NW.m: h = 0.5, lambda = 1e-3 when both are unset)
    const double bw = lw->bandwidth > 0 ? lw->bandwidth : (D->bandwidth > 0 ? D->bandwidth : 0.5);
    const double lam = lw->lambda > 0 ? lw->lambda : (D->lambda > 0 ? D->lambda : 1e-3);
    bqp_lbmpc_dims dl = *d;
    dl.mask = 1;                          // the loop's window always carries the validity row
    bqp_lbmpc_data Dl = *D;
    Dl.data = win; Dl.sdata = (int64_t)q * 8;
    Dl.x0 = s; Dl.sx0 = nx;
    Dl.bin = bin; Dl.sbin = m;
    Dl.bandwidth = bw; Dl.lambda = lam;
    EventGuard e0;
    HIP_TRY(hipEventCreate(&e0.e));
    HIP_TRY(hipEventRecord(e0.e, st));
    int launches = 0;
    // BQP_LB_SYNC selects the step-synchronous loop below (the asynchronous loop's bitwise
    // reference in tests/test_gpu_lbmpc_dms.py); BQP_LB_TRACE only adds diagnostics to either
    const bool sync_loop = getenv("BQP_LB_SYNC") != nullptr;
    if (!sync_loop) {
        // asynchronous (round 5): every instance runs at its own closed-loop step.  Each round is
        // one SQP iteration of every unfinished instance, then sqp_loop_advance_kernel moves the
        // instances whose SQP has finished to their next step (u_0, plant, window, constraints,
        // warm start).  The step-synchronous form below ran every step's SQP launches until the
        // batch's slowest instance had converged (2.4 SQP iterations per step on average against
        // up to 6 at a step) while the converged ones idled; per instance the two forms do the
        // same operations in the same order (tests/test_gpu_lbmpc_dms.py compares them).
        int* ts = it + B;
        int* nfin = ts + B;
        HIP_TRY(hipMemsetAsync(ts, 0, sizeof(int) * (B + 1), st));
        HIP_TRY(bqp::launch_sqp_loop_prep(batch, nx, n, m, N * d->nu, 0, s, sl->bin0, sl->Bx, bin, z, st));
        bqp::LbmpcArgs a;
        bqp::DenseKernelArgs qd;
        HIP_TRY(lbmpc_setup(h, &dl, batch, &Dl, *opt, z, nullptr, fl, it, st, a, qd));
        // sub-problem polish per instance: from its own SQP iteration count (lbmpc solve: mode 2
        // from LB_POLISH_STALL on, before it the loop's mode 3 - none - or 1)
        qd.polish = opt->polish < 0 ? 0 : (opt->polish == 3 ? 0 : 1);
        qd.pol_it = opt->polish < 0 ? nullptr : a.iters;
        qd.pol_stall = LB_POLISH_STALL;
        bqp::SqpAdvanceArgs v;
        memset(&v, 0, sizeof(v));
        v.batch = batch; v.nx = nx; v.nu = d->nu; v.n = n; v.m = m; v.nv = N * d->nu; v.warm = sl->warm;
        v.steps = cl->steps; v.q = q; v.plant = cl->plant; v.delta = cl->delta;
        v.hinv2 = 1.0 / (bw * bw); v.lam = lam;
        v.K = D->K; v.bin0 = sl->bin0; v.Bx = sl->Bx; v.xeq = cl->x_eq; v.ueq = cl->u_eq;
        v.A = D->A; v.Bm = D->B;
        v.s = s; v.z = z; v.bin = bin; v.X = X; v.U = U; v.win = win; v.XL = lw->XL; v.Zlog = sl->Z;
        v.done = a.done; v.iters = a.iters; v.flag = fl; v.hused = a.hused; v.ts = ts; v.nfin = nfin;
        v.flags = exitflag; v.itlog = sl->iterations;
        const int max_rounds = cl->steps * opt->max_iter;
        for (int r = 0; r < max_rounds; ++r) {
            HIP_TRY(bqp::launch_lbmpc_rollout(a, 1, st));
            HIP_TRY(bqp::launch_lbmpc_normal(a, st));
            if (a.hess) HIP_TRY(bqp::launch_lbmpc_hess(a, st));
            HIP_TRY(bqp::launch_dense(qd, st));
            HIP_TRY(bqp::launch_lbmpc_rollout(a, 0, st));
            HIP_TRY(bqp::launch_lbmpc_update(a, st));
            HIP_TRY(bqp::launch_sqp_loop_advance(v, st));
            launches += a.hess ? 7 : 6;
            int nf = 0;
            HIP_TRY(hipMemcpyAsync(&nf, nfin, sizeof(int), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (nf >= batch) break;
        }
    }
    for (int t = 0; t < (sync_loop ? cl->steps : 0); ++t) {
        HIP_TRY(bqp::launch_sqp_loop_prep(batch, nx, n, m, N * d->nu, t > 0 && sl->warm, s,
                                          sl->bin0, sl->Bx, bin, z, st));
        if (t > 0 && !sl->warm) HIP_TRY(hipMemsetAsync(z, 0, sizeof(double) * B * n, st));
        rc = bqp_lbmpc_solve_batched_device(h, &dl, batch, &Dl, opt, z, nullptr, nullptr, fl, it,
                                            stream);
        if (rc) return rc;
        launches += h->launches;
        HIP_TRY(bqp::launch_sqp_loop_u0(batch, nx, n, D->K, s, z, uo, it, cl->steps, t,
                                        sl->Z, sl->iterations, st));
        HIP_TRY(bqp::launch_mg_plant(cl->plant, batch, 1, cl->steps, t, cl->delta, uo, fl, cl->x_eq, cl->u_eq,
                                     s, X, U, exitflag, st));
        HIP_TRY(bqp::launch_lbmpc_window(batch, cl->steps, t, q, bw, lam, D->A, 0, D->B, 0,
                                         cl->x_eq, cl->u_eq, X, U, win, lw->XL, st));
        launches += 3;
    }
    HIP_TRY(hipEventRecord(h->ev1, st));
    HIP_TRY(hipEventSynchronize(h->ev1));
    std::swap(h->ev0, e0.e);   // the guard destroys the previous start event
    h->timed = true;
    h->launches = launches;
    return BQP_OK;
}

int bqp_closed_loop_sqp(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                        const bqp_lbmpc_data* D, const bqp_sqp_loop* sl, const bqp_options* opt,
                        const bqp_closed_loop* cl, const bqp_learning* lw, const double* x_init,
                        double* X, double* U, int* exitflag) {
    if (!h) return BQP_E_ARG;
    int rc = sqp_loop_check(d, batch, D, sl, cl, lw, x_init, X, U);
    if (rc) return rc;
    DevScope ds(h->device);
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N, m = d->m, q = d->q;
    const int n = N * nu + np;
    struct In { const double* src; size_t n; double* dst; };
    In in[] = {
        {D->A, (size_t)nx * nx, nullptr}, {D->B, (size_t)nx * nu, nullptr},
        {D->K, (size_t)nu * nx, nullptr}, {D->Lq, (size_t)nx * nx, nullptr},
        {D->Lr, (size_t)nu * nu, nullptr}, {D->Lp, (size_t)nx * nx, nullptr},
        {D->Lt, (size_t)nx * nx, nullptr}, {D->LAMBDA, (size_t)nx * np, nullptr},
        {D->PSI, (size_t)nu * np, nullptr}, {D->xs, (size_t)nx, nullptr},
        {D->Ain, (size_t)m * n, nullptr}, {sl->bin0, (size_t)m, nullptr},
        {sl->Bx, (size_t)m * nx, nullptr}, {x_init, (size_t)batch * nx, nullptr},
        {cl->x_eq, (size_t)nx, nullptr}, {cl->u_eq, (size_t)nu, nullptr},
    };
    const int nin = sizeof(in) / sizeof(in[0]);
    const size_t B = batch, S = cl->steps;
    const size_t nX = B * (S + 1) * nx, nU = B * S * nu, nW = B * (size_t)q * 8, nZ = B * S * n;
    size_t tot = 2 * nX + nU + nW + (sl->Z ? nZ : 0);
    for (int i = 0; i < nin; ++i) tot += (in[i].src ? in[i].n : 0);
    HIP_TRY(h->stage.reserve(sizeof(double) * tot + sizeof(int) * 2 * B * S));
    double* cur = (double*)h->stage.p;
    for (int i = 0; i < nin; ++i) {
        if (!in[i].src || in[i].n == 0) continue;
        in[i].dst = cur;
        HIP_TRY(hipMemcpyAsync(cur, in[i].src, sizeof(double) * in[i].n, hipMemcpyHostToDevice, h->stream));
        cur += in[i].n;
    }
    double* Xd = cur; cur += nX;
    double* Ud = cur; cur += nU;
    double* XLd = cur; cur += nX;
    double* Wd = cur; cur += nW;
    double* Zd = nullptr;
    if (sl->Z) { Zd = cur; cur += nZ; }
    int* Fd = (int*)cur;
    int* Id = Fd + B * S;
    bqp_lbmpc_data Dd = *D;
    Dd.A = in[0].dst; Dd.B = in[1].dst; Dd.K = in[2].dst; Dd.Lq = in[3].dst; Dd.Lr = in[4].dst;
    Dd.Lp = in[5].dst; Dd.Lt = in[6].dst; Dd.LAMBDA = in[7].dst; Dd.PSI = in[8].dst;
    Dd.xs = in[9].dst; Dd.Ain = in[10].dst;
    bqp_sqp_loop sd = *sl;
    sd.bin0 = in[11].dst; sd.Bx = in[12].dst;
    sd.Z = Zd; sd.iterations = sl->iterations ? Id : nullptr;
    bqp_closed_loop cd = *cl;
    cd.x_eq = in[14].dst; cd.u_eq = in[15].dst;
    bqp_learning ld = *lw;
    ld.XL = XLd; ld.window = Wd;
    rc = bqp_closed_loop_sqp_device(h, d, batch, &Dd, &sd, opt, &cd, &ld, in[13].dst, Xd, Ud,
                                    exitflag ? Fd : nullptr, h->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(X, Xd, sizeof(double) * nX, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(U, Ud, sizeof(double) * nU, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(lw->XL, XLd, sizeof(double) * nX, hipMemcpyDeviceToHost, h->stream));
    if (lw->window) HIP_TRY(hipMemcpyAsync(lw->window, Wd, sizeof(double) * nW, hipMemcpyDeviceToHost, h->stream));
    if (sl->Z) HIP_TRY(hipMemcpyAsync(sl->Z, Zd, sizeof(double) * nZ, hipMemcpyDeviceToHost, h->stream));
    if (exitflag) HIP_TRY(hipMemcpyAsync(exitflag, Fd, sizeof(int) * B * S, hipMemcpyDeviceToHost, h->stream));
    if (sl->iterations) HIP_TRY(hipMemcpyAsync(sl->iterations, Id, sizeof(int) * B * S, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return BQP_OK;
}

#ifdef BQP_STAMPS
// diagnostic build only: per-instance phase cycle counts of the last structured solve
// (32 per instance: 16 stage-wave phases, 16 row-wave phases)
int bqp_debug_stamps(bqp_handle h, int N, int nv, int mp, double* out) {
    if (!h || !out) return BQP_E_ARG;
    DevScope ds(h->device);
    const int hstride = nv * nv + 1;
    const int mpad = 64 * bqp::ocp_rpl_for(std::max(mp, 1));
    const size_t off = (size_t)(N + 1) * hstride + (size_t)nv * mpad + (size_t)h->last_batch * bqp::STATS_W + 8;
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, (double*)h->work.p + off, sizeof(double) * h->last_batch * 32, hipMemcpyDeviceToHost));
    return BQP_OK;
}
#endif

}  // extern "C"
