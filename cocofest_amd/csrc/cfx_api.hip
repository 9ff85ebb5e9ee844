// cfx_api.hip — the C ABI of libcfx (include/cfx.h): problem set-up on the host, stimulation
// coefficient tables, sparsity, buffer staging, and the launches of the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cfx.h"
#include "cfx_aux.h"
#include "cfx_colloc.h"
#include "cfx_internal.h"
#include "cfx_launch.h"
#include "cfx_msk_launch.h"

using namespace cfx;

// last failure of a handle-free call (cfx_create, cfx_band_lu*) on this thread; cfx_last_error(NULL)
thread_local std::string g_create_error;

namespace {

enum Slot { S_V = 0, S_A1, S_A2, S_G, S_J, S_F, S_GRAD, S_OUT, S_WORK, S_COUNT };

struct DevBuf {
    double* p = nullptr;
    size_t n = 0;
};

}  // namespace

struct cfx_handle {
    cfx_problem prob{};
    std::vector<double> rows;
    std::vector<int32_t> last_idx;
    std::vector<cfx_objective> objs;
    cfx_sizes sz{};
    int model = 0, scheme = 1, tmax = 1, stages = 1, ni = 1, ni_g = 1;
    bool colloc = false;  // direct collocation (n_steps = polynomial degree)
    double tau[kMaxDeg + 1] = {};
    int32_t* d_hdiag = nullptr;
    KParams kp{};
    int device = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    double* d_tab = nullptr;
    double* d_rest = nullptr;
    double* d_cna = nullptr;
    DevObjective* d_obj = nullptr;
    double* d_targets = nullptr;
    int32_t* d_sl_param = nullptr;
    int32_t* d_sl_joff = nullptr;
    HTask* d_htasks = nullptr;
    int n_htasks = 1, hbs = 1;
    int n_obj = 0;
    std::vector<int32_t> jrow, jcol, hrow, hcol;
    // J_g values that depend on neither the instance nor the point (cfx_jac_constant_mask), and whether the handle's
    // own J_g staging buffer (AoS / host outputs) holds them from an earlier full evaluation
    std::vector<uint8_t> jconst;
    bool jconst_staged = false;
    // musculoskeletal problems (cfx_msk_create)
    bool msk = false;
    int msk_nq = 0, msk_nm = 0, msk_fam = 0;
    // stage-data reuse between cfx_eval_all (with J_g) and the next cfx_eval_h at the same caller pointer, while the
    // interior point (the only caller that guarantees the point is unchanged in between) has it switched on
    bool msk_stash = false, stash_valid = false, stash_same_point = false;
    MskParams mp{};
    MskGeom* d_geom = nullptr;
    MskObjective* d_mobj = nullptr;
    double* d_msk_imin = nullptr;  // Hmed: I_min per muscle (sliding-window padding)
    int msk_ns = 0;                // Hmed: sliding-window rows per interval (0: none)
    MskMarker* d_mk = nullptr;     // marker superimpositions (cfx_msk_marker_pair)
    int n_mk = 0;
    int32_t* d_ties = nullptr;     // CFX_MSK_PULSE_WIDTH_PER_PULSE: rows v[a] - v[b], [n_ties][2]
    int n_ties = 0;
    int64_t tie_row0 = 0, tie_j0 = 0;  // their first g row and J_g value
    double* d_cs1 = nullptr;       // CFX_MSK_LEGACY_CALCIUM: d cs / d Km per stage and muscle
    DevBuf main[S_COUNT], stage[S_COUNT];
    std::string err;
};

#define CFX_HIP(h, call)                                                                      \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            (h)->err = std::string(#call) + ": " + hipGetErrorString(e_);                     \
            return CFX_EHIP;                                                                  \
        }                                                                                     \
    } while (0)

static int fail(cfx_handle* h, int code, const std::string& msg) {
    h->err = msg;
    return code;
}

// ------------------------------------------------------------------------------------------------------
// stimulation coefficients (cocofest/models/ding2003.py:200-252; hmed2018.py:97-98)
// ------------------------------------------------------------------------------------------------------
static double legendre_p(int n, double x) {
    if (n == 0) return 1.0;
    double p0 = 1.0, p1 = x;
    for (int k = 2; k <= n; ++k) {
        const double p2 = ((2.0 * k - 1.0) * x * p1 - (k - 1.0) * p0) / k;
        p0 = p1;
        p1 = p2;
    }
    return p1;
}

// Collocation points on (0, 1]: Gauss-Legendre (roots of P_d) or Radau IIA (roots of P_d - P_{d-1}, x = 1
// included), mapped from [-1, 1]; sign-change scan + bisection to machine precision.  Then the Lagrange basis
// through tau_0 = 0 and the points: C[i][j] = l_i'(tau_j), D[i] = l_i(1).
static void collocation_coefficients(int d, bool radau, double* tau, double (*C)[kMaxDeg + 1], double* D) {
    auto f = [&](double x) { return radau ? legendre_p(d, x) - legendre_p(d - 1, x) : legendre_p(d, x); };
    int found = 0;
    const int M = 40000;
    double xa = -1.0, fa = f(xa);
    for (int i = 1; i <= M && found < d; ++i) {
        const double xb = -1.0 + 2.0 * i / M;
        if (radau && i == M) break;  // the root x = 1 is added below
        const double fb = f(xb);
        if (fb == 0.0) {
            tau[1 + found++] = xb;
        } else if (fa * fb < 0.0) {
            double lo = xa, hi = xb, flo = fa;
            for (int it = 0; it < 200 && hi - lo > 0.0; ++it) {
                const double mid = 0.5 * (lo + hi);
                if (mid == lo || mid == hi) break;
                const double fm = f(mid);
                if ((fm < 0.0) == (flo < 0.0)) {
                    lo = mid;
                    flo = fm;
                } else {
                    hi = mid;
                }
            }
            tau[1 + found++] = 0.5 * (lo + hi);
        }
        xa = xb;
        fa = fb;
    }
    if (radau) tau[1 + found++] = 1.0;
    tau[0] = 0.0;
    for (int j = 1; j <= d; ++j) tau[j] = (tau[j] + 1.0) / 2.0;
    for (int i = 0; i <= d; ++i) {
        double den = 1.0, num1 = 1.0;
        for (int r = 0; r <= d; ++r)
            if (r != i) {
                den *= tau[i] - tau[r];
                num1 *= 1.0 - tau[r];
            }
        D[i] = num1 / den;
        for (int j = 0; j <= d; ++j) {
            double v;
            if (j == i) {
                v = 0.0;
                for (int r = 0; r <= d; ++r)
                    if (r != i) v += 1.0 / (tau[i] - tau[r]);
            } else {
                v = 1.0 / (tau[i] - tau[j]);
                for (int r = 0; r <= d; ++r)
                    if (r != i && r != j) v *= (tau[j] - tau[r]) / (tau[i] - tau[r]);
            }
            C[i][j] = v;
        }
    }
}

// Calcium sums (Ding) / per-stimulus coefficients (Hmed) at the collocation points t_k + tau_j dt,
// slot k*d + j - 1 — the same expression and operation order as the RK stage tables.
static void build_colloc_tables(const cfx_handle* h, std::vector<double>& tab) {
    const cfx_problem& p = h->prob;
    const cfx_constants& c = p.constants;
    const int N = p.n_shooting, d = p.n_steps, T = p.truncation;
    const double dt = p.final_time / N;
    const double r0 = c.km_rest + c.r0_km_relationship;
    const bool hmed = is_int(h->model);
    const int w = hmed ? h->tmax : 1;
    tab.assign((size_t)N * d * w, 0.0);
    std::vector<double> ri(T);
    for (int k = 0; k < N; ++k) {
        const double* row = &h->rows[(size_t)k * T];
        for (int i = 0; i < T; ++i) ri[i] = i == 0 ? 1.0 : 1.0 + (r0 - 1.0) * std::exp(-(row[i] - row[i - 1]) / c.tauc);
        for (int j = 1; j <= d; ++j) {
            const double t = k * dt + h->tau[j] * dt;
            const size_t q = (size_t)k * d + j - 1;
            if (hmed) {
                for (int i = 0; i < T; ++i) tab[q * w + i] = ri[i] * std::exp(-(t - row[i]) / c.tauc);
            } else {
                double sum = 0.0;
                for (int i = 0; i < T; ++i) sum = sum + ri[i] * std::exp(-(t - row[i]) / c.tauc);
                tab[q] = sum;
            }
        }
    }
}

static void build_tables(const cfx_handle* h, std::vector<double>& tab) {
    const cfx_problem& p = h->prob;
    const cfx_constants& c = p.constants;
    const int N = p.n_shooting, m = p.n_steps, T = p.truncation, S = h->stages;
    const double dt = p.final_time / N;
    const double hh = dt / m;
    const double r0 = c.km_rest + c.r0_km_relationship;
    const bool hmed = is_int(h->model);
    const int Q = m * S;
    tab.assign((size_t)N * Q * (hmed ? h->tmax : 1), 0.0);
    std::vector<double> ri(T);
    for (int k = 0; k < N; ++k) {
        const double* row = &h->rows[(size_t)k * T];
        for (int i = 0; i < T; ++i) ri[i] = i == 0 ? 1.0 : 1.0 + (r0 - 1.0) * std::exp(-(row[i] - row[i - 1]) / c.tauc);
        const double t0 = k * dt;
        for (int j = 0; j < m; ++j) {
            const double tj = t0 + j * hh;
            for (int s = 0; s < S; ++s) {
                double t = tj;
                if (S == 2 && s == 1) t = tj + hh / 2;
                if (S == 4 && (s == 1 || s == 2)) t = tj + hh / 2;
                if (S == 4 && s == 3) t = tj + hh;
                const size_t q = (size_t)k * Q + (size_t)j * S + s;
                if (hmed) {
                    for (int i = 0; i < T; ++i) tab[q * h->tmax + i] = ri[i] * std::exp(-(t - row[i]) / c.tauc);
                } else {
                    double sum = 0.0;
                    for (int i = 0; i < T; ++i) sum = sum + ri[i] * std::exp(-(t - row[i]) / c.tauc);
                    tab[q] = sum;
                }
            }
        }
    }
}

// Dependency bitmask (over z = (x_k, u_k)) of every state after one interval (bits 0..nx-1: states,
// nx..nx+nu-1: controls).  RHS dependencies: cn_dot <- cn (+ every Hmed intensity through cn_sum);
// F_dot <- cn, F (+ A, Tau1, Km with fatigue, + pulse width for Ding2007); A/Tau1/Km_dot <- itself, F.
static void structure_pattern(int model, int scheme, int m, int nx, int nu, uint64_t* dep) {
    const bool fat = is_fatigue(model), pw = is_pw(model), hm = is_int(model);
    const uint64_t ubits = hm ? (((1ull << nu) - 1ull) << nx) : 0ull;
    const uint64_t pwbit = pw ? (1ull << nx) : 0ull;
    auto f = [&](const uint64_t* x, uint64_t* o) {
        o[0] = x[0] | ubits;
        o[1] = x[0] | x[1] | (fat ? (x[2] | x[3] | x[4]) : 0ull) | pwbit;
        if (fat) {
            o[2] = x[2] | x[1];
            o[3] = x[3] | x[1];
            o[4] = x[4] | x[1];
        }
    };
    uint64_t x[5], k[5], xs[5], acc[5];
    for (int r = 0; r < nx; ++r) x[r] = 1ull << r;
    for (int j = 0; j < m; ++j) {
        f(x, k);
        if (scheme == 1) {
            for (int r = 0; r < nx; ++r) x[r] |= k[r];
            continue;
        }
        for (int r = 0; r < nx; ++r) {
            acc[r] = k[r];
            xs[r] = x[r] | k[r];
        }
        const int extra = scheme == 2 ? 1 : 3;
        for (int st = 0; st < extra; ++st) {
            f(xs, k);
            for (int r = 0; r < nx; ++r) {
                acc[r] |= k[r];
                xs[r] = x[r] | k[r];
            }
        }
        for (int r = 0; r < nx; ++r) x[r] |= acc[r];
    }
    for (int r = 0; r < nx; ++r) dep[r] = x[r];
}

// Ding families: the calcium state under explicit RK is affine in the interval start value,
// cn(slot) = cna[slot] * cn0 + cnb[k][slot] (see cfx_kernels.h, integrate).  Derived from the stage-time
// calcium sums cs[k*Q + slot] by running the scheme on (slope, offset) pairs.
static void affine_calcium(const cfx_handle* h, const std::vector<double>& cs, std::vector<double>& cna,
                           std::vector<double>& cnb) {
    const int N = h->prob.n_shooting, m = h->prob.n_steps, S = h->stages, Q = m * S;
    const double al = 1.0 / h->prob.constants.tauc;
    const double hh = (h->prob.final_time / N) / m;
    cna.assign(Q + 1, 0.0);
    cnb.assign((size_t)N * (Q + 1), 0.0);
    for (int k = 0; k < N; ++k) {
        double a = 1.0, b = 0.0;
        double* ob = &cnb[(size_t)k * (Q + 1)];
        auto rate = [&](double sa, double sb, int q, double& ka, double& kb) {  // k = al (cs - cn)
            ka = -al * sa;
            kb = al * (cs[(size_t)k * Q + q] - sb);
        };
        for (int j = 0; j < m; ++j) {
            const int q = j * S;
            cna[q] = a;
            ob[q] = b;
            double k1a, k1b;
            rate(a, b, q, k1a, k1b);
            if (S == 1) {
                a += hh * k1a;
                b += hh * k1b;
            } else if (S == 2) {
                const double sa = a + hh / 2 * k1a, sb = b + hh / 2 * k1b;
                cna[q + 1] = sa;
                ob[q + 1] = sb;
                double k2a, k2b;
                rate(sa, sb, q + 1, k2a, k2b);
                a += hh * k2a;
                b += hh * k2b;
            } else {
                double sa = a + hh / 2 * k1a, sb = b + hh / 2 * k1b, k2a, k2b, k3a, k3b, k4a, k4b;
                cna[q + 1] = sa;
                ob[q + 1] = sb;
                rate(sa, sb, q + 1, k2a, k2b);
                sa = a + hh / 2 * k2a;
                sb = b + hh / 2 * k2b;
                cna[q + 2] = sa;
                ob[q + 2] = sb;
                rate(sa, sb, q + 2, k3a, k3b);
                sa = a + hh * k3a;
                sb = b + hh * k3b;
                cna[q + 3] = sa;
                ob[q + 3] = sb;
                rate(sa, sb, q + 3, k4a, k4b);
                a += hh / 6 * (k1a + 2 * k2a + 2 * k3a + k4a);
                b += hh / 6 * (k1b + 2 * k2b + 2 * k3b + k4b);
            }
        }
        cna[Q] = a;
        ob[Q] = b;
    }
}

static double* ensure(cfx_handle* h, DevBuf& b, size_t count, int* rc) {
    if (b.n < count) {
        if (b.p) (void)hipFree(b.p);
        b.p = nullptr;
        b.n = 0;
        hipError_t e = hipMalloc((void**)&b.p, count * sizeof(double));
        if (e != hipSuccess) {
            h->err = std::string("hipMalloc: ") + hipGetErrorString(e);
            *rc = CFX_ENOMEM;
            return nullptr;
        }
        b.n = count;
    }
    return b.p;
}

// transposes: 64 x 64 tiles, the element tiles strided over grid.y (a per-instance length past 64 * 65535 loops)
static dim3 tgrid(int64_t B, int64_t len) {
    return dim3((unsigned)((B + 63) / 64), (unsigned)std::min<int64_t>((len + 63) / 64, kMaxGridY));
}

// AoS buffers go through a transpose unless they are SoA already: one element per instance, or one instance
// (a batch of 1 has the same memory image in both layouts).
static bool is_aos(const cfx_handle* h, int64_t len) {
    return h->prob.layout == CFX_LAYOUT_AOS && len > 1 && h->prob.batch > 1;
}

// Device SoA view of an input buffer of `len` doubles per instance.
static const double* stage_in(cfx_handle* h, int slot, const double* ptr, int64_t len, uint32_t flags, int* rc) {
    const int64_t B = h->prob.batch;
    const bool dev = flags & CFX_DEVICE;
    const bool aos = is_aos(h, len);
    if (dev && !aos) return ptr;
    const size_t n = (size_t)B * len;
    double* m = ensure(h, h->main[slot], n, rc);
    if (!m) return nullptr;
    const double* src = ptr;
    if (!dev) {
        double* target = aos ? ensure(h, h->stage[slot], n, rc) : m;
        if (!target) return nullptr;
        if (hipMemcpyAsync(target, ptr, n * sizeof(double), hipMemcpyHostToDevice, h->stream) != hipSuccess) {
            *rc = CFX_EHIP;
            h->err = "hipMemcpyAsync H2D failed";
            return nullptr;
        }
        if (!aos) return m;
        src = target;
    }
    hipLaunchKernelGGL(k_aos_to_soa, tgrid(B, len), dim3(256), 0, h->stream, src, m, B, len);
    return m;
}

// Device SoA buffer an output is written to.
static double* stage_out(cfx_handle* h, int slot, double* ptr, int64_t len, uint32_t flags, int* rc) {
    const bool dev = flags & CFX_DEVICE;
    const bool aos = is_aos(h, len);
    if (dev && !aos) return ptr;
    return ensure(h, h->main[slot], (size_t)h->prob.batch * len, rc);
}

static int finish_out(cfx_handle* h, int slot, double* soa, double* ptr, int64_t len, uint32_t flags) {
    const int64_t B = h->prob.batch;
    const bool dev = flags & CFX_DEVICE;
    const bool aos = is_aos(h, len);
    const size_t n = (size_t)B * len;
    if (dev && !aos) return CFX_OK;
    double* src = soa;
    if (aos) {
        int rc = CFX_OK;
        double* dst = dev ? ptr : ensure(h, h->stage[slot], n, &rc);
        if (!dst) return rc;
        hipLaunchKernelGGL(k_soa_to_aos, tgrid(B, len), dim3(256), 0, h->stream, soa, dst, B, len);
        if (dev) return CFX_OK;
        src = dst;
    }
    CFX_HIP(h, hipMemcpyAsync(ptr, src, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    return CFX_OK;
}

static int sync_if_host(cfx_handle* h, uint32_t flags) {
    if (!(flags & CFX_DEVICE)) CFX_HIP(h, hipStreamSynchronize(h->stream));
    CFX_HIP(h, hipGetLastError());
    return CFX_OK;
}

// ------------------------------------------------------------------------------------------------------
// lifetime
// ------------------------------------------------------------------------------------------------------
static int create_fail(cfx_handle* h, int code, const std::string& msg) {
    g_create_error = msg;
    if (h) cfx_destroy(h);
    return code;
}

extern "C" int cfx_abi_version(void) { return CFX_ABI_VERSION; }

extern "C" int cfx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int cfx_create(const cfx_problem* p, cfx_handle** out) {
    if (!p || !out) return create_fail(nullptr, CFX_EINVAL, "cfx_create: NULL argument");
    *out = nullptr;
    if (p->abi_version != CFX_ABI_VERSION) return create_fail(nullptr, CFX_EINVAL, "cfx_create: ABI version mismatch");
    if (p->model < CFX_DING2003 || p->model > CFX_HMED2018_FATIGUE)
        return create_fail(nullptr, CFX_EINVAL, "cfx_create: unknown model");
    const bool colloc = p->scheme == CFX_COLLOCATION_LEGENDRE || p->scheme == CFX_COLLOCATION_RADAU;
    if (p->scheme != CFX_RK1 && p->scheme != CFX_RK2 && p->scheme != CFX_RK4 && !colloc)
        return create_fail(nullptr, CFX_EUNSUPPORTED,
                           "cfx_create: scheme must be CFX_RK1, CFX_RK2, CFX_RK4 or CFX_COLLOCATION_LEGENDRE/RADAU");
    if (colloc && (p->n_steps < 1 || p->n_steps > kMaxDeg))
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_create: collocation degree (n_steps) must be in [1, 9]");
    if (p->n_steps < 1 || p->n_shooting < 1 || p->batch < 1 || !(p->final_time > 0.0))
        return create_fail(nullptr, CFX_EINVAL, "cfx_create: n_steps, n_shooting, batch and final_time must be positive");
    if (p->truncation < 1 || p->truncation > 32)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_create: truncation must be in [1, 32]");
    if (p->layout != CFX_LAYOUT_AOS && p->layout != CFX_LAYOUT_SOA && p->layout != CFX_LAYOUT_TILED64)
        return create_fail(nullptr, CFX_EINVAL, "cfx_create: unknown layout");
    if (p->layout == CFX_LAYOUT_TILED64 && p->batch % 64 != 0)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_create: CFX_LAYOUT_TILED64 needs batch % 64 == 0");
    if (!p->stim_rows) return create_fail(nullptr, CFX_EINVAL, "cfx_create: stim_rows is NULL");
    if (p->n_objectives < 0 || (p->n_objectives > 0 && !p->objectives))
        return create_fail(nullptr, CFX_EINVAL, "cfx_create: n_objectives < 0, or objectives is NULL");
    if (p->n_shooting > kMaxGridY)  // grid.y = intervals in the shooting / Hessian / collocation launches
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_create: n_shooting must be <= 65535");
    const bool hmed = p->model >= CFX_HMED2018;
    if (p->n_params < 0 || (p->n_params > 0 && (!hmed || !p->last_stim_idx)))
        return create_fail(nullptr, CFX_EINVAL,
                           "cfx_create: intensity parameters need a Hmed2018 model and last_stim_idx");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return create_fail(nullptr, CFX_ENODEV, "cfx_create: no HIP device available (libcfx has no CPU path)");
    if (p->device < 0 || p->device >= ndev) return create_fail(nullptr, CFX_ENODEV, "cfx_create: bad device ordinal");

    cfx_handle* h = new cfx_handle();
    h->prob = *p;
    h->model = p->model;
    h->scheme = p->scheme;
    h->stages = colloc ? 1 : stages_of(p->scheme);
    h->colloc = colloc;
    h->device = p->device;
    const int N = p->n_shooting, T = p->truncation;
    h->rows.assign(p->stim_rows, p->stim_rows + (size_t)(N + 1) * T);
    if (p->n_params > 0) {
        h->last_idx.assign(p->last_stim_idx, p->last_stim_idx + N);
        for (int k = 0; k < N; ++k)
            if (h->last_idx[k] >= p->n_params)
                return create_fail(h, CFX_EINVAL, "cfx_create: last_stim_idx out of the parameter range");
    }
    h->prob.stim_rows = nullptr;
    h->prob.last_stim_idx = nullptr;
    h->tmax = hmed ? tmax_bucket(T) : 1;

    const int nx = is_fatigue(h->model) ? 5 : 2;
    const int nu = is_pw(h->model) ? 1 : (hmed ? T : 0);
    const int deg = colloc ? p->n_steps : 0;
    const int uoff = colloc ? (deg + 1) * nx : nx;
    const int nz = uoff + nu;  // decision block of one interval
    const int n_slide = (hmed && p->n_params > 0) ? T : 0;
    const int ngk = (colloc ? (deg + 1) * nx : nx) + n_slide;

    // objectives
    std::vector<DevObjective> dobj;
    std::vector<double> targets;
    for (int t = 0; t < p->n_objectives; ++t) {
        const cfx_objective& o = p->objectives[t];
        const bool st = o.var_kind == CFX_VAR_STATE;
        const int lim = st ? N : N - 1;
        if ((o.var_kind != CFX_VAR_STATE && o.var_kind != CFX_VAR_CONTROL) || o.var_index < 0 ||
            o.var_index >= (st ? nx : nu) || o.node_first < 0 || o.node_last > lim || o.node_first > o.node_last ||
            (o.kind != CFX_OBJ_LAGRANGE && o.kind != CFX_OBJ_MAYER))
            return create_fail(h, CFX_EINVAL, "cfx_create: invalid objective term " + std::to_string(t));
        DevObjective d{};
        d.var_kind = st ? 0 : 1;
        d.var_index = o.var_index;
        d.node_first = o.node_first;
        d.node_last = o.node_last;
        d.w_eff = o.weight * (o.kind == CFX_OBJ_LAGRANGE ? p->final_time / N : 1.0);
        d.target_value = o.target_value;
        d.target_off = -1;
        if (o.target) {
            d.target_off = (int32_t)targets.size();
            targets.insert(targets.end(), o.target, o.target + N + 1);
        }
        dobj.push_back(d);
    }
    h->n_obj = (int)dobj.size();
    h->prob.objectives = nullptr;

    // sizes + sparsity
    h->sz.nx = nx;
    h->sz.nu = nu;
    h->sz.nv = (int64_t)N * nz + nx + p->n_params;
    h->sz.ng = (int64_t)N * ngk;
    const int per_point = nx * (nx + 1) / 2 + nu * nx;  // collocation Hessian entries of one point
    const int nhk = colloc ? nx + deg * per_point + nu * (nu + 1) / 2 : nz * (nz + 1) / 2;
    KParams& kp = h->kp;
    int nnzk = 0;
    std::vector<uint8_t> ccst;  // collocation: constant J_g values, in triplet order
    if (!colloc) {
        // structural sparsity of dPhi/d(x_k, u_k), as CasADi derives it symbolically: dependency bitmasks
        // pushed through the RHS and the RK stages (identical for every interval)
        uint64_t dep[5];
        structure_pattern(h->model, h->scheme, p->n_steps, nx, nu, dep);
        for (int r = 0; r < nx; ++r) {
            for (int c = 0; c < kMaxNz; ++c) kp.jpos[r][c] = -1;
            for (int c = 0; c < nz; ++c)
                if (dep[r] >> c & 1ull) kp.jpos[r][c] = (int16_t)nnzk++;
            kp.jneg[r] = (int16_t)nnzk++;
        }
        for (int k = 0; k < N; ++k) {
            for (int r = 0; r < nx; ++r) {
                for (int c = 0; c < nz; ++c) {
                    if (!(dep[r] >> c & 1ull)) continue;
                    h->jrow.push_back(k * ngk + r);
                    h->jcol.push_back(k * nz + c);
                }
                h->jrow.push_back(k * ngk + r);
                h->jcol.push_back((k + 1) * nz + r);
            }
        }
    } else {
        // collocation (cfx_colloc.h): defect rows [x^0_r..x^d_r, other states of point j, controls], then
        // continuity rows [x^0_r..x^d_r, -1 on x_{k+1}^0_r].  Constant values (ccst): the basis coefficients C[i][j]
        // off the point's own state, the whole calcium row (its right-hand side (cs - cn) / tau_c is linear in cn),
        // every continuity value D[i] and -1
        for (int k = 0; k < N; ++k) {
            const size_t before = h->jrow.size();
            auto put = [&](int row, int col, bool cst) {
                h->jrow.push_back(row);
                h->jcol.push_back(col);
                ccst.push_back(cst);
            };
            for (int j = 1; j <= deg; ++j)
                for (int r = 0; r < nx; ++r) {
                    const int row = k * ngk + (j - 1) * nx + r;
                    for (int i = 0; i <= deg; ++i) put(row, k * nz + i * nx + r, r == 0 || i != j);
                    for (int c = 0; c < nx; ++c)
                        if (c != r && (col_xdeps(h->model, r) >> c & 1u)) put(row, k * nz + j * nx + c, false);
                    for (int c = 0; c < col_udeps(h->model, r, nu); ++c) put(row, k * nz + uoff + c, false);
                }
            for (int r = 0; r < nx; ++r) {
                const int row = k * ngk + deg * nx + r;
                for (int i = 0; i <= deg; ++i) put(row, k * nz + i * nx + r, true);
                put(row, (k + 1) * nz + r, true);
            }
            nnzk = (int)(h->jrow.size() - before);
        }
    }
    std::vector<int32_t> sl_param, sl_joff;
    const int p_off = N * nz + nx;
    if (n_slide) {
        for (int k = 0; k < N; ++k) {
            const int idx = h->last_idx[k];
            const int first = idx + 1 - T;
            for (int j = 0; j < T; ++j) {
                const int pi = first + j;
                const bool valid = pi >= 0 && pi <= idx;
                sl_param.push_back(valid ? pi : -1);
                sl_joff.push_back((int32_t)h->jrow.size());
                h->jrow.push_back(k * ngk + (ngk - n_slide) + j);
                h->jcol.push_back(k * nz + uoff + j);
                if (valid) {
                    h->jrow.push_back(k * ngk + (ngk - n_slide) + j);
                    h->jcol.push_back(p_off + pi);
                }
            }
        }
    }
    h->sz.nnz_jac = (int64_t)h->jrow.size();
    // constant J_g values: the -1 on x_{k+1} of every continuity row and, for the Ding families (calcium affine in
    // its start value, cfx_kernels.h:integrate), dCn+/dCn0 = cna[m S]
    h->jconst.assign(h->jrow.size(), 0);
    std::copy(ccst.begin(), ccst.end(), h->jconst.begin());
    if (!colloc)
        for (int k = 0; k < N; ++k) {
            for (int r = 0; r < nx; ++r) h->jconst[(size_t)k * nnzk + kp.jneg[r]] = 1;
            if (!is_int(h->model) && kp.jpos[0][0] >= 0) h->jconst[(size_t)k * nnzk + kp.jpos[0][0]] = 1;
        }
    auto hput = [&](int r, int c) {
        h->hrow.push_back(r);
        h->hcol.push_back(c);
    };
    std::vector<int32_t> hdiag((size_t)(N + 1) * (nx + nu), -1);  // objective-term diagonal positions
    for (int k = 0; k < N; ++k) {
        if (!colloc) {
            for (int i = 0; i < nz; ++i) {
                hdiag[(size_t)k * (nx + nu) + i] = (int32_t)(k * nhk + i * (i + 1) / 2 + i);
                for (int j = 0; j <= i; ++j) hput(k * nz + i, k * nz + j);
            }
        } else {
            for (int r = 0; r < nx; ++r) {
                hdiag[(size_t)k * (nx + nu) + r] = (int32_t)(k * nhk + r);
                hput(k * nz + r, k * nz + r);
            }
            for (int j = 1; j <= deg; ++j) {
                for (int a = 0; a < nx; ++a)
                    for (int b = 0; b <= a; ++b) hput(k * nz + j * nx + a, k * nz + j * nx + b);
                for (int a = 0; a < nu; ++a)
                    for (int b = 0; b < nx; ++b) hput(k * nz + uoff + a, k * nz + j * nx + b);
            }
            for (int a = 0; a < nu; ++a) {
                hdiag[(size_t)k * (nx + nu) + nx + a] = (int32_t)(k * nhk + nx + deg * per_point + a * (a + 1) / 2 + a);
                for (int b = 0; b <= a; ++b) hput(k * nz + uoff + a, k * nz + uoff + b);
            }
        }
    }
    for (int r = 0; r < nx; ++r) {
        hdiag[(size_t)N * (nx + nu) + r] = (int32_t)(N * nhk + r);
        hput(N * nz + r, N * nz + r);
    }
    h->sz.nnz_hess = (int64_t)h->hrow.size();

    // kernel parameters
    const cfx_constants& c = p->constants;
    kp.B = p->batch;
    kp.tiled = p->layout == CFX_LAYOUT_TILED64;
    kp.nv_tot = h->sz.nv;
    kp.ng_tot = h->sz.ng;
    kp.nnz_tot = h->sz.nnz_jac;
    kp.nh_tot = h->sz.nnz_hess;
    kp.nx = nx;
    kp.N = N;
    kp.m = p->n_steps;
    kp.nu = nu;
    kp.nz = nz;
    kp.T = T;
    kp.Q = colloc ? deg : p->n_steps * h->stages;
    kp.uoff = uoff;
    kp.deg = deg;
    if (colloc) collocation_coefficients(deg, p->scheme == CFX_COLLOCATION_RADAU, h->tau, kp.colC, kp.colD);
    kp.ngk = ngk;
    kp.nnzk = nnzk;
    kp.nhk = nhk;
    kp.n_slide = n_slide;
    kp.n_params = p->n_params;
    kp.dt = p->final_time / N;
    kp.h = kp.dt / p->n_steps;
    kp.inv_tauc = 1.0 / c.tauc;
    kp.tau2 = c.tau2;
    kp.km_rest = c.km_rest;
    kp.tau1_rest = c.tau1_rest;
    kp.a_rest = c.a_rest;
    kp.a_scale = c.a_scale;
    kp.pd0 = c.pd0;
    kp.pdt = c.pdt;
    kp.ar = c.ar;
    kp.bs = c.bs;
    kp.Is = c.Is;
    kp.cr = c.cr;
    kp.alpha_a = c.alpha_a;
    kp.alpha_tau1 = c.alpha_tau1;
    kp.alpha_km = c.alpha_km;
    kp.inv_tau_fat = is_fatigue(h->model) ? 1.0 / c.tau_fat : 0.0;
    kp.a_fat_rest = is_pw(h->model) ? c.a_scale : c.a_rest;
    kp.mult = c.fl * c.fv + c.fp;
    kp.neg_mult = -kp.mult;
    kp.mult_km = kp.mult * c.km_rest;
    kp.tau12 = c.tau1_rest + c.tau2;
    kp.tau1km = c.tau1_rest * c.km_rest;
    kp.hm = kp.h * kp.mult;
    kp.hmkm = kp.hm * c.km_rest;
    kp.hmkmt2 = kp.hmkm * c.tau2;
    {
        // instances per thread (Ding families): 2 side by side once the batch fills the chip twice over;
        // CFX_NI=1|2|4 overrides (tuning)
        // NI adjacent instances per lane (16-byte accesses) need B % NI == 0; the launch also checks alignment
        // Measured on MI355X (cfg2, B = 2^20): g + J_g is store-bound and fastest at NI = 1; the g-only pass
        // (fewer stores) gains ~7% from NI = 4.
        // With 64-instance tiles the g + J_g pass is fastest at NI = 2 (0.29 vs 0.30 ms at NI = 1, SoA NI = 1:
        // 0.32 ms; scripts/kprobe.py).
        h->ni = (!hmed && p->layout == CFX_LAYOUT_TILED64) ? 2 : 1;
        // collocation (degrees 1..5, Ding families): two instances per lane whenever the batch pairs up
        if (colloc) h->ni = (!hmed && deg <= 5 && p->batch % 2 == 0) ? 2 : 1;
        h->ni_g = (!hmed && p->batch % 4 == 0 && p->batch >= (int64_t)256 * 1024) ? 4 : 1;
        if (const char* e = std::getenv("CFX_NI")) {
            const int v = std::atoi(e);
            if (!hmed && (v == 1 || v == 2 || v == 4) && p->batch % v == 0) h->ni = h->ni_g = v;
        }
        if (colloc && (hmed || deg > 5 || h->ni > 2)) h->ni = h->ni_g = 1;  // what the collocation kernels run
        // intervals per thread: about 40 workgroups per CU (10,240).  Longer chunks read fewer boundary states
        // twice but start every wave in the same phase; cfg 2 at B = 2^20 (20 intervals, 2,048 instance blocks):
        // 0.313 / 0.304 / 0.295 / 0.287 / 0.293 / 0.303 ms at 20 / 10 / 5 / 4 / 2 / 1 intervals per thread
        // (scripts/store_probe.py).
        const int64_t bx = (p->batch + (int64_t)kBlock * h->ni - 1) / ((int64_t)kBlock * h->ni);
        const int64_t nch = colloc ? 1 : nchunk_of(h->model, h->scheme, h->tmax, nz);
        int64_t kpt = (int64_t)N * bx * nch / 10240;
        kp.kpt = (int32_t)std::max<int64_t>(1, std::min<int64_t>(N, kpt));
        if (const char* e = std::getenv("CFX_KPT"))  // tuning override
            kp.kpt = (int32_t)std::max<int64_t>(1, std::min<int64_t>(N, std::atoi(e)));
        // interval chunks as the fast grid index, so the chunks of one instance block — one region of each output
        // tile — are dispatched together (0.296 -> 0.287 ms above); the instance blocks must then fit grid.y.
        // CFX_IFAST=0|1 overrides (tuning).
        kp.ifast = bx <= kMaxGridY;
        if (const char* e = std::getenv("CFX_IFAST"))
            kp.ifast = std::atoi(e) != 0 && bx <= kMaxGridY;
    }

    if (hipSetDevice(h->device) != hipSuccess) return create_fail(h, CFX_EHIP, "cfx_create: hipSetDevice failed");
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess)
        return create_fail(h, CFX_EHIP, "cfx_create: hipStreamCreate failed");
    h->stream = h->own_stream;

    std::vector<double> tab, cna;
    if (colloc) {
        build_colloc_tables(h, tab);
        kp.tstride = deg;
    } else {
        build_tables(h, tab);
    }
    if (colloc) {
    } else if (!hmed) {
        std::vector<double> cnb;
        affine_calcium(h, tab, cna, cnb);
        tab.swap(cnb);
        kp.tstride = kp.Q + 1;
    } else {
        kp.tstride = kp.Q;
    }
    std::vector<double> rest(nx, 0.0);
    if (nx == 5) {
        rest[2] = kp.a_fat_rest;
        rest[3] = c.tau1_rest;
        rest[4] = c.km_rest;
    }
    // Hessian tasks: blocks of bs directions, one task per block pair (I <= J); a single task when the
    // lane's jet holds every direction
    std::vector<HTask> htasks;
    {
        const int dj = hjet_of(h->model);
        h->hbs = hsplit_of(h->model) ? dj / 2 : dj;
        const int ndir = colloc ? nx + nu : nz;  // collocation: directions of one point (x^j, u)
        const int nb = (ndir + h->hbs - 1) / h->hbs;
        for (int I = 0; I < nb; ++I)
            for (int J = I; J < nb; ++J) htasks.push_back(HTask{(int16_t)I, (int16_t)J});
        h->n_htasks = (int)htasks.size();
        if (!hsplit_of(h->model) && nb != 1)
            return create_fail(h, CFX_EINVAL, "cfx_create: internal Hessian task layout error");
    }
    auto upload = [&](void** dst, const void* src, size_t bytes) -> bool {
        if (bytes == 0) return true;
        if (hipMalloc(dst, bytes) != hipSuccess) return false;
        return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!upload((void**)&h->d_tab, tab.data(), tab.size() * sizeof(double)) ||
        !upload((void**)&h->d_rest, rest.data(), rest.size() * sizeof(double)) ||
        !upload((void**)&h->d_cna, cna.data(), cna.size() * sizeof(double)) ||
        !upload((void**)&h->d_obj, dobj.data(), dobj.size() * sizeof(DevObjective)) ||
        !upload((void**)&h->d_targets, targets.data(), targets.size() * sizeof(double)) ||
        !upload((void**)&h->d_sl_param, sl_param.data(), sl_param.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_sl_joff, sl_joff.data(), sl_joff.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_htasks, htasks.data(), htasks.size() * sizeof(HTask)) ||
        !upload((void**)&h->d_hdiag, hdiag.data(), hdiag.size() * sizeof(int32_t)))
        return create_fail(h, CFX_ENOMEM, "cfx_create: device allocation/upload failed");
    kp.tab = h->d_tab;
    kp.cna = h->d_cna;
    kp.rest = h->d_rest;
    kp.hdiag = h->d_hdiag;
    *out = h;
    return CFX_OK;
}

extern "C" void cfx_destroy(cfx_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (int s = 0; s < S_COUNT; ++s) {
        if (h->main[s].p) (void)hipFree(h->main[s].p);
        if (h->stage[s].p) (void)hipFree(h->stage[s].p);
    }
    for (void* p : {(void*)h->d_tab, (void*)h->d_rest, (void*)h->d_cna, (void*)h->d_htasks, (void*)h->d_obj,
                    (void*)h->d_targets, (void*)h->d_sl_param, (void*)h->d_sl_joff, (void*)h->d_hdiag,
                    (void*)h->d_geom, (void*)h->d_mobj, (void*)h->d_msk_imin, (void*)h->d_mk, (void*)h->d_ties,
                    (void*)h->d_cs1})
        if (p) (void)hipFree(p);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
}

extern "C" int cfx_get_sizes(const cfx_handle* h, cfx_sizes* out) {
    if (!h || !out) return CFX_EINVAL;
    *out = h->sz;
    return CFX_OK;
}

extern "C" int cfx_get_launch_shape(const cfx_handle* h, cfx_launch_shape* out) {
    if (!h || !out) return CFX_EINVAL;
    std::memset(out, 0, sizeof(*out));
    if (h->msk) {
        out->msk_intervals_per_block = h->mp.kpb;
    } else {
        out->intervals_per_thread = h->kp.kpt;
        out->intervals_fast = h->kp.ifast;
        out->instances_per_lane = h->ni;
        out->instances_per_lane_g = h->ni_g;
    }
    return CFX_OK;
}

// internal (cfx_internal.h): what the interior-point driver needs to know about a handle
int cfx_internal_info(const cfx_handle* h, int64_t* batch, int* layout, int* device, hipStream_t* stream) {
    if (!h) return CFX_EINVAL;
    *batch = h->prob.batch;
    *layout = h->prob.layout;
    *device = h->device;
    *stream = h->stream;
    return CFX_OK;
}

extern "C" int cfx_set_stream(cfx_handle* h, void* stream) {
    if (!h) return CFX_EINVAL;
    h->stream = (hipStream_t)stream;
    return CFX_OK;
}

extern "C" int cfx_synchronize(cfx_handle* h) {
    if (!h) return CFX_EINVAL;
    CFX_HIP(h, hipStreamSynchronize(h->stream));
    return CFX_OK;
}

extern "C" const char* cfx_last_error(const cfx_handle* h) { return h ? h->err.c_str() : g_create_error.c_str(); }

extern "C" int cfx_jac_structure(const cfx_handle* h, int32_t* row, int32_t* col) {
    if (!h || !row || !col) return CFX_EINVAL;
    std::memcpy(row, h->jrow.data(), h->jrow.size() * sizeof(int32_t));
    std::memcpy(col, h->jcol.data(), h->jcol.size() * sizeof(int32_t));
    return CFX_OK;
}

extern "C" int cfx_hess_structure(const cfx_handle* h, int32_t* row, int32_t* col) {
    if (!h || !row || !col) return CFX_EINVAL;
    std::memcpy(row, h->hrow.data(), h->hrow.size() * sizeof(int32_t));
    std::memcpy(col, h->hcol.data(), h->hcol.size() * sizeof(int32_t));
    return CFX_OK;
}

// ------------------------------------------------------------------------------------------------------
// evaluation
// ------------------------------------------------------------------------------------------------------
static hipError_t launch_shooting(cfx_handle* h, bool derivs, const double* V, double* G, double* J, bool keep) {
    // 16-byte lane accesses need 16-byte aligned buffers (B % NI == 0 keeps every row aligned)
    auto aligned = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    KParams kp = h->kp;
    kp.keepc = keep ? 1 : 0;
    if (h->colloc) {
        const int ni = (aligned(V) && aligned(G) && aligned(J)) ? h->ni : 1;
        return launch_colloc(h->model, h->tmax, ni, kp, V, G, derivs ? J : nullptr, h->stream);
    }
    if (is_int(h->model)) return launch_shooting_hmed(h->model, h->scheme, derivs, h->tmax, kp, V, G, J, h->stream);
    const int ni = (aligned(V) && aligned(G) && aligned(J)) ? (derivs ? h->ni : h->ni_g) : 1;
    return launch_shooting_ding(h->model, h->scheme, derivs, ni, kp, V, G, J, h->stream);
}

// CFX_KEEP_CONSTANT_JAC: skip the constant J_g values when the buffer the kernels write holds them — the caller's
// buffer on the direct device path (the caller's contract), the handle's staging buffer once a full evaluation has
// filled it.  Whether the next staged evaluation may skip is recorded here.
static bool keep_constants(cfx_handle* h, uint32_t flags, const double* J) {
    if (!J) return false;
    const bool staged = !(flags & CFX_DEVICE) || is_aos(h, h->sz.nnz_jac);
    const bool keep = (flags & CFX_KEEP_CONSTANT_JAC) && (!staged || h->jconst_staged);
    if (staged) h->jconst_staged = true;
    return keep;
}

extern "C" int cfx_jac_constant_mask(const cfx_handle* h, uint8_t* mask) {
    if (!h || !mask) return CFX_EINVAL;
    std::memcpy(mask, h->jconst.data(), h->jconst.size());
    return CFX_OK;
}

// Hmed sliding-window rows of g / J_g (k_slide; nothing for the other families)
static void launch_slide(cfx_handle* h, const double* V, double* G, double* J) {
    if (!h->kp.n_slide) return;
    const int64_t B = h->prob.batch;
    hipLaunchKernelGGL(k_slide,
                       dim3((unsigned)((B + 255) / 256),
                            (unsigned)std::min<int64_t>((int64_t)h->kp.N * h->kp.T, kMaxGridY)),
                       dim3(256), 0, h->stream, h->kp, h->d_sl_param, h->d_sl_joff, h->prob.intensity_floor, V, G, J);
}

// f and grad f (either may be NULL)
static hipError_t launch_objective(cfx_handle* h, const double* V, double* F, double* GR) {
    const int64_t B = h->prob.batch;
    if ((F || GR) && B < kObjBlockMaxB) {  // latency-bound: a block per instance, a thread per node
        hipLaunchKernelGGL(k_objective_blk, dim3((unsigned)B), dim3(256), 0, h->stream, h->kp, h->n_obj, h->d_obj,
                           h->d_targets, V, F, GR);
    } else if (F || GR) {
        if (GR) {
            hipError_t e = hipMemsetAsync(GR, 0, (size_t)B * h->sz.nv * sizeof(double), h->stream);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_objective, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, h->stream, h->kp, h->n_obj,
                           h->d_obj, h->d_targets, V, F, GR);
    }
    return hipGetLastError();
}

// obj_factor * Hess(f) added onto the constraint Hessian H
static hipError_t launch_objective_hess(cfx_handle* h, const double* OF, double* H) {
    const int64_t B = h->prob.batch;
    if (h->n_obj && B < kObjBlockMaxB)
        hipLaunchKernelGGL(k_objective_hess_blk, dim3((unsigned)B), dim3(256), 0, h->stream, h->kp, h->n_obj,
                           h->d_obj, OF, H);
    else if (h->n_obj)
        hipLaunchKernelGGL(k_objective_hess, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, h->stream, h->kp,
                           h->n_obj, h->d_obj, OF, H);
    return hipGetLastError();
}

static int msk_eval_all(cfx_handle* h, const double* v, double* g, double* jac, double* f, double* grad,
                        uint32_t flags);
static int msk_eval_h(cfx_handle* h, const double* v, const double* obj_factor, const double* lambda, double* hess,
                      uint32_t flags);
static int msk_integrate(cfx_handle* h, const double* x0, const double* u, double* traj, uint32_t flags);

extern "C" int cfx_eval_all(cfx_handle* h, const double* v, double* g, double* jac, double* f, double* grad,
                            uint32_t flags) {
    if (!h || !v) return CFX_EINVAL;
    if (h->msk) return msk_eval_all(h, v, g, jac, f, grad, flags);
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const double* V = stage_in(h, S_V, v, h->sz.nv, flags, &rc);
    if (!V) return rc;
    double* G = g ? stage_out(h, S_G, g, h->sz.ng, flags, &rc) : nullptr;
    double* J = jac ? stage_out(h, S_J, jac, h->sz.nnz_jac, flags, &rc) : nullptr;
    double* F = f ? stage_out(h, S_F, f, 1, flags, &rc) : nullptr;
    double* GR = grad ? stage_out(h, S_GRAD, grad, h->sz.nv, flags, &rc) : nullptr;
    if (rc != CFX_OK) return rc;
    if (G || J) {
        CFX_HIP(h, launch_shooting(h, J != nullptr, V, G, J, keep_constants(h, flags, J)));
        launch_slide(h, V, G, J);
    }
    CFX_HIP(h, launch_objective(h, V, F, GR));
    if (G && (rc = finish_out(h, S_G, G, g, h->sz.ng, flags)) != CFX_OK) return rc;
    if (J && (rc = finish_out(h, S_J, J, jac, h->sz.nnz_jac, flags)) != CFX_OK) return rc;
    if (F && (rc = finish_out(h, S_F, F, f, 1, flags)) != CFX_OK) return rc;
    if (GR && (rc = finish_out(h, S_GRAD, GR, grad, h->sz.nv, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

extern "C" int cfx_eval_g(cfx_handle* h, const double* v, double* g, uint32_t flags) {
    if (!g) return h ? fail(h, CFX_EINVAL, "cfx_eval_g: g is NULL") : CFX_EINVAL;
    return cfx_eval_all(h, v, g, nullptr, nullptr, nullptr, flags);
}

extern "C" int cfx_eval_jac_g(cfx_handle* h, const double* v, double* jac, uint32_t flags) {
    if (!jac) return h ? fail(h, CFX_EINVAL, "cfx_eval_jac_g: jac is NULL") : CFX_EINVAL;
    return cfx_eval_all(h, v, nullptr, jac, nullptr, nullptr, flags);
}

extern "C" int cfx_eval_f(cfx_handle* h, const double* v, double* f, uint32_t flags) {
    if (!f) return h ? fail(h, CFX_EINVAL, "cfx_eval_f: f is NULL") : CFX_EINVAL;
    return cfx_eval_all(h, v, nullptr, nullptr, f, nullptr, flags);
}

extern "C" int cfx_eval_grad_f(cfx_handle* h, const double* v, double* grad, uint32_t flags) {
    if (!grad) return h ? fail(h, CFX_EINVAL, "cfx_eval_grad_f: grad is NULL") : CFX_EINVAL;
    return cfx_eval_all(h, v, nullptr, nullptr, nullptr, grad, flags);
}

extern "C" int cfx_eval_h(cfx_handle* h, const double* v, const double* obj_factor, const double* lambda,
                          double* hess, uint32_t flags) {
    if (!h || !v || !obj_factor || !lambda || !hess) return h ? fail(h, CFX_EINVAL, "cfx_eval_h: NULL argument") : CFX_EINVAL;
    if (h->msk) return msk_eval_h(h, v, obj_factor, lambda, hess, flags);
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const double* V = stage_in(h, S_V, v, h->sz.nv, flags, &rc);
    if (!V) return rc;
    const double* OF = stage_in(h, S_A1, obj_factor, 1, flags, &rc);
    if (!OF) return rc;
    const double* LAM = stage_in(h, S_A2, lambda, h->sz.ng, flags, &rc);
    if (!LAM) return rc;
    double* H = stage_out(h, S_OUT, hess, h->sz.nnz_hess, flags, &rc);
    if (!H) return rc;
    if (h->colloc)
        CFX_HIP(h, launch_colloc_hess(h->model, h->tmax, h->kp, h->d_htasks, h->n_htasks, h->hbs, V, LAM, H, nullptr,
                                      nullptr, h->stream));
    else
        CFX_HIP(h, launch_hessian(h->model, h->scheme, h->tmax, h->kp, h->d_htasks, h->n_htasks, h->hbs, V, LAM, H,
                                  nullptr, nullptr, h->stream));
    CFX_HIP(h, launch_objective_hess(h, OF, H));
    if ((rc = finish_out(h, S_OUT, H, hess, h->sz.nnz_hess, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

extern "C" int cfx_eval_all_h(cfx_handle* h, const double* v, const double* obj_factor, const double* lambda,
                              double* g, double* jac, double* f, double* grad, double* hess, uint32_t flags) {
    if (!h || !v || !obj_factor || !lambda || !g || !jac || !hess)
        return h ? fail(h, CFX_EINVAL, "cfx_eval_all_h: NULL argument") : CFX_EINVAL;
    if (h->msk) {  // the callbacks, then the Hessian at the same point
        int rc = cfx_eval_all(h, v, g, jac, f, grad, flags);
        if (rc != CFX_OK) return rc;
        if (h->msk) h->stash_same_point = h->msk_stash && h->stash_valid;
        return cfx_eval_h(h, v, obj_factor, lambda, hess, flags);
    }
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const double* V = stage_in(h, S_V, v, h->sz.nv, flags, &rc);
    if (!V) return rc;
    const double* OF = stage_in(h, S_A1, obj_factor, 1, flags, &rc);
    if (!OF) return rc;
    const double* LAM = stage_in(h, S_A2, lambda, h->sz.ng, flags, &rc);
    if (!LAM) return rc;
    double* G = stage_out(h, S_G, g, h->sz.ng, flags, &rc);
    double* J = stage_out(h, S_J, jac, h->sz.nnz_jac, flags, &rc);
    double* F = f ? stage_out(h, S_F, f, 1, flags, &rc) : nullptr;
    double* GR = grad ? stage_out(h, S_GRAD, grad, h->sz.nv, flags, &rc) : nullptr;
    double* H = stage_out(h, S_OUT, hess, h->sz.nnz_hess, flags, &rc);
    if (rc != CFX_OK || !G || !J || !H) return rc != CFX_OK ? rc : fail(h, CFX_EINVAL, "cfx_eval_all_h: staging");
    // one launch: shooting — the interval's second-order jets carry the g rows and the J_g columns too; collocation
    // — task 0 of every interval runs the g + J_g body (defects, continuity) beside its Hessian block
    KParams kp = h->kp;
    kp.keepc = keep_constants(h, flags, J) ? 1 : 0;
    if (h->colloc)
        CFX_HIP(h, launch_colloc_hess(h->model, h->tmax, kp, h->d_htasks, h->n_htasks, h->hbs, V, LAM, H, G, J,
                                      h->stream));
    else
        CFX_HIP(h, launch_hessian(h->model, h->scheme, h->tmax, kp, h->d_htasks, h->n_htasks, h->hbs, V, LAM, H, G, J,
                                  h->stream));
    launch_slide(h, V, G, J);
    CFX_HIP(h, launch_objective(h, V, F, GR));
    CFX_HIP(h, launch_objective_hess(h, OF, H));
    if ((rc = finish_out(h, S_G, G, g, h->sz.ng, flags)) != CFX_OK) return rc;
    if ((rc = finish_out(h, S_J, J, jac, h->sz.nnz_jac, flags)) != CFX_OK) return rc;
    if (F && (rc = finish_out(h, S_F, F, f, 1, flags)) != CFX_OK) return rc;
    if (GR && (rc = finish_out(h, S_GRAD, GR, grad, h->sz.nv, flags)) != CFX_OK) return rc;
    if ((rc = finish_out(h, S_OUT, H, hess, h->sz.nnz_hess, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

extern "C" int cfx_integrate(cfx_handle* h, const double* x0, const double* u, double* traj, uint32_t flags) {
    if (!h || !traj) return CFX_EINVAL;
    if (h->msk) return msk_integrate(h, x0, u, traj, flags);
    if (h->colloc) return fail(h, CFX_EUNSUPPORTED, "cfx_integrate: not available for a collocation transcription");
    if (h->kp.tiled) return fail(h, CFX_EUNSUPPORTED, "cfx_integrate: not available with CFX_LAYOUT_TILED64");
    if (h->sz.nu > 0 && !u) return fail(h, CFX_EINVAL, "cfx_integrate: this model needs per-interval controls");
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const int64_t nsamp = (int64_t)h->kp.N * h->kp.m + 1;
    const double* X0 = x0 ? stage_in(h, S_A1, x0, h->sz.nx, flags, &rc) : nullptr;
    if (x0 && !X0) return rc;
    const double* U = h->sz.nu ? stage_in(h, S_A2, u, (int64_t)h->kp.N * h->sz.nu, flags, &rc) : nullptr;
    if (h->sz.nu && !U) return rc;
    double* TR = stage_out(h, S_OUT, traj, nsamp * h->sz.nx, flags, &rc);
    if (!TR) return rc;
    hipError_t e = is_int(h->model) ? launch_ivp_hmed(h->model, h->scheme, h->tmax, h->kp, X0, U, TR, h->stream)
                                    : launch_ivp_ding(h->model, h->scheme, h->kp, X0, U, TR, h->stream);
    CFX_HIP(h, e);
    if ((rc = finish_out(h, S_OUT, TR, traj, nsamp * h->sz.nx, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

// ------------------------------------------------------------------------------------------------------
// musculoskeletal problems (FesMskModel + OcpFesMsk; cfx_msk.h)
// ------------------------------------------------------------------------------------------------------
int cfx_internal_msk_stash(cfx_handle* h, int on) {
    if (!h) return CFX_EINVAL;
    if (on == 2) {  // the caller vouches that the next eval_h is at the point of the last eval_all with J_g
        h->stash_same_point = h->msk_stash && h->stash_valid;
        return CFX_OK;
    }
    h->msk_stash = h->msk && on;
    h->stash_valid = h->stash_same_point = false;
    return CFX_OK;
}

extern "C" int cfx_msk_create(const cfx_msk_problem* p, cfx_handle** out) {
    if (!p || !out) return create_fail(nullptr, CFX_EINVAL, "cfx_msk_create: NULL argument");
    *out = nullptr;
    auto bad = [](const std::string& m) { return create_fail(nullptr, CFX_EINVAL, "cfx_msk_create: " + m); };
    if (p->abi_version != CFX_ABI_VERSION) return bad("ABI version mismatch");
    if (p->scheme != CFX_RK1 && p->scheme != CFX_RK2 && p->scheme != CFX_RK4)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_msk_create: scheme must be CFX_RK1, CFX_RK2 or CFX_RK4");
    if (p->n_steps < 1 || p->n_shooting < 1 || p->batch < 1 || !(p->final_time > 0.0))
        return bad("n_steps, n_shooting, batch and final_time must be positive");
    if (p->truncation < 1 || p->truncation > 64) return bad("truncation must be in [1, 64]");
    if (p->n_shooting > kMaxGridY)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_msk_create: n_shooting must be <= 65535");
    if (p->n_objectives < 0 || (p->n_objectives > 0 && !p->objectives))
        return bad("n_objectives < 0, or objectives is NULL");
    if (p->layout != CFX_LAYOUT_AOS && p->layout != CFX_LAYOUT_SOA)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_msk_create: layout must be CFX_LAYOUT_AOS or CFX_LAYOUT_SOA");
    if (!p->stim_rows || !p->dof_axis || !p->dof_frame || !p->body_mass || !p->body_com || !p->body_inertia ||
        !p->muscles)
        return bad("NULL array");
    const int nq = p->n_dof, nm = p->n_muscles;
    if (nq < 1 || nq > CFX_MSK_MAX_DOF) return bad("n_dof must be in [1, 4]");
    if (nm < 1 || nm > CFX_MSK_MAX_MUSCLES) return bad("n_muscles must be in [1, 8]");
    const int model = p->muscles[0].model;
    if (model < CFX_DING2003 || model > CFX_HMED2018_FATIGUE)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_msk_create: unknown muscle model");
    const bool hmed = model >= CFX_HMED2018;
    if (hmed && p->truncation > 20)
        return create_fail(nullptr, CFX_EUNSUPPORTED, "cfx_msk_create: Hmed2018 muscles need truncation <= 20");
    // kernel family: Ding 0..3 as the model ids; Hmed2018 4 / 5 (T <= 10) and 6 / 7 (T <= 20), bit 0 fatigue
    const int fam = hmed ? 4 + (model - CFX_HMED2018) + (p->truncation > 10 ? 2 : 0) : model;
    if (p->n_params < 0 || (p->n_params > 0 && (!hmed || !p->last_stim_idx || !p->param_offset)))
        return bad("intensity parameters need Hmed2018 muscles, last_stim_idx and param_offset");
    if ((p->flags & CFX_MSK_LEGACY_CALCIUM) && hmed) return bad("CFX_MSK_LEGACY_CALCIUM needs Ding2003 / Ding2007 muscles");
    if ((p->flags & CFX_MSK_PULSE_WIDTH_PER_PULSE) && !(model == CFX_DING2007 || model == CFX_DING2007_FATIGUE))
        return bad("CFX_MSK_PULSE_WIDTH_PER_PULSE needs Ding2007 muscles (pulse-width controls)");
    for (int m = 0; m < nm; ++m) {
        const cfx_msk_muscle& mu = p->muscles[m];
        if (mu.model != model) return bad("every muscle must use the same model family");
        if (mu.n_points < 2 || mu.n_points > CFX_MSK_MAX_POINTS || !mu.point_frame || !mu.point_pos)
            return bad("muscle " + std::to_string(m) + ": 2..16 path points with frames and positions");
        for (int i = 0; i < mu.n_points; ++i)
            if (mu.point_frame[i] < -1 || mu.point_frame[i] >= nq) return bad("muscle point frame out of range");
        if (!(mu.optimal_length > 0.0) || !(std::cos(mu.pennation_angle) > 0.0))
            return bad("muscle optimal length must be positive and |pennation| < pi/2");
    }
    for (int j = 0; j < nq; ++j)
        if (p->dof_axis[j] < 0 || p->dof_axis[j] > 2) return bad("dof_axis must be 0, 1 or 2");
    if (p->n_marker_pairs < 0 || (p->n_marker_pairs > 0 && !p->marker_pairs))
        return bad("n_marker_pairs < 0, or marker_pairs is NULL");
    for (int i = 0; i < p->n_marker_pairs; ++i) {
        const cfx_msk_marker_pair& c = p->marker_pairs[i];
        if (c.node < 0 || c.node > p->n_shooting) return bad("marker pair node out of [0, n_shooting]");
        if (c.axes < 1 || c.axes > 7) return bad("marker pair axes must select X, Y and / or Z (bits 1, 2, 4)");
        for (int e = 0; e < 2; ++e)
            if (c.frame[e] < -1 || c.frame[e] >= nq) return bad("marker frame out of range");
        if (c.frame[0] < 0 && c.frame[1] < 0) return bad("marker pair: both markers are fixed to the ground");
    }
    if (!msk_supported(nq, nm, fam, p->scheme))
        return create_fail(nullptr, CFX_EUNSUPPORTED,
                           "cfx_msk_create: shape (n_dof " + std::to_string(nq) + ", muscles " + std::to_string(nm) +
                               ", model " + std::to_string(fam) + ", scheme " + std::to_string(p->scheme) +
                               ") is not compiled into this libcfx (cfx_inst_msk_*.hip)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return create_fail(nullptr, CFX_ENODEV, "cfx_msk_create: no HIP device available (libcfx has no CPU path)");
    if (p->device < 0 || p->device >= ndev) return create_fail(nullptr, CFX_ENODEV, "cfx_msk_create: bad device ordinal");

    const bool fat = model & 1, pw = model == CFX_DING2007 || model == CFX_DING2007_FATIGUE;
    const bool residual = p->flags & CFX_MSK_RESIDUAL_TORQUE;
    const int N = p->n_shooting, T = p->truncation, m = p->n_steps, S = stages_of(p->scheme);
    const int nxm = fat ? 5 : 2, nx = nm * nxm + 2 * nq, npw = pw ? nm : 0, nint = hmed ? nm * T : 0;
    const int nu = npw + nint + (residual ? nq : 0);
    const int nz = nx + nu;
    if (nz > 64) return bad("more than 64 decision variables per interval");
    const int ns = p->n_params > 0 ? nint : 0;  // sliding-window rows per interval
    const int ngk = nx + ns;
    if (p->n_params > 0) {
        for (int k = 0; k < N; ++k)
            if (p->last_stim_idx[k] < -1) return bad("last_stim_idx out of range");
        for (int mi = 0; mi < nm; ++mi) {
            const int64_t hi = (int64_t)p->param_offset[mi] + p->last_stim_idx[N - 1];
            if (p->param_offset[mi] < 0 || hi >= p->n_params) return bad("param_offset / last_stim_idx out of range");
        }
    }

    cfx_handle* h = new cfx_handle();
    h->msk = true;
    h->msk_nq = nq, h->msk_nm = nm, h->msk_fam = fam;
    h->prob.abi_version = p->abi_version;
    h->prob.scheme = p->scheme, h->prob.n_steps = m, h->prob.n_shooting = N, h->prob.truncation = T;
    h->prob.layout = p->layout, h->prob.batch = p->batch, h->prob.final_time = p->final_time;
    h->prob.device = p->device;
    h->scheme = p->scheme, h->stages = S, h->device = p->device;

    // ---- constants
    // Every joint turned into a rotation about its frame's z axis, so the kernels carry no per-joint axis selects:
    // frame j is replaced by R'_j = R_j P_j, whose columns are R_j's columns perm_j = (a, b, axis) — (1, 2, 0) for x,
    // (2, 0, 1) for y, (0, 1, 2) for z — and R_j Rot_axis(q) P_j = R_j P_j Rot_z(q).  Quantities given in frame j
    // follow: p' = P_j^T p (com, via points, markers), I' = P_j^T I P_j, and the constant joint transform becomes
    // A'_j = P_{j-1}^T A_j P_j, t'_j = P_{j-1}^T t_j (P_{-1} = I, the ground).  World positions, axes, the mass
    // matrix and every callback value are unchanged.
    int perm[kMskMaxQ + 1][3];  // perm[j + 1]: frame j (perm[0]: the ground)
    for (int e = 0; e < 3; ++e) perm[0][e] = e;
    for (int j = 0; j < nq; ++j) {
        const int ax = p->dof_axis[j];
        for (int e = 0; e < 3; ++e) perm[j + 1][e] = (ax + 1 + e) % 3;
    }
    auto pf = [&](int frame) { return perm[frame + 1]; };  // frame -1: the ground
    MskGeom G;
    std::memset(&G, 0, sizeof(G));
    for (int j = 0; j < nq; ++j) {
        const int *pp = pf(j - 1), *pj = pf(j);
        G.axis[j] = 2;
        for (int r = 0; r < 3; ++r)
            for (int c2 = 0; c2 < 3; ++c2) G.A[j][r * 3 + c2] = p->dof_frame[j * 12 + pp[r] * 3 + pj[c2]];
        for (int e = 0; e < 3; ++e) G.t[j][e] = p->dof_frame[j * 12 + 9 + pp[e]];
        G.mass[j] = p->body_mass[j];
        for (int e = 0; e < 3; ++e) G.com[j][e] = p->body_com[j * 3 + pj[e]];
        for (int r = 0; r < 3; ++r)
            for (int c2 = 0; c2 < 3; ++c2) G.inertia[j][r * 3 + c2] = p->body_inertia[j * 9 + pj[r] * 3 + pj[c2]];
    }
    for (int e = 0; e < 3; ++e) G.grav[e] = p->gravity[e];
    std::vector<double> rest(nx, 0.0);
    for (int mi = 0; mi < nm; ++mi) {
        const cfx_msk_muscle& mu = p->muscles[mi];
        const cfx_constants& c = mu.constants;
        // A path segment whose two ends are fixed in the same frame keeps its length and adds nothing to the
        // length Jacobian (d . (z x d) = 0): its length is summed once here; the kernels visit only the segments
        // that cross frames (2 of the 8 of BIClong, 2 of the 4 of TRIlong in arm26).
        int ns = 0;
        double cl = 0.0;
        for (int i = 0; i + 1 < mu.n_points; ++i) {
            const double* a = mu.point_pos + i * 3;
            const double* e3 = mu.point_pos + (i + 1) * 3;
            if (mu.point_frame[i] == mu.point_frame[i + 1]) {
                cl += std::sqrt((e3[0] - a[0]) * (e3[0] - a[0]) + (e3[1] - a[1]) * (e3[1] - a[1]) +
                                (e3[2] - a[2]) * (e3[2] - a[2]));
                continue;
            }
            G.seg_frame[mi][ns][0] = mu.point_frame[i];
            G.seg_frame[mi][ns][1] = mu.point_frame[i + 1];
            const int *p0 = pf(mu.point_frame[i]), *p1 = pf(mu.point_frame[i + 1]);
            for (int e = 0; e < 3; ++e) {
                G.seg_pos[mi][ns][0][e] = a[p0[e]];
                G.seg_pos[mi][ns][1][e] = e3[p1[e]];
            }
            ++ns;
        }
        G.nseg[mi] = ns;
        G.const_len[mi] = cl;
        MskMuscleConst& C = G.mc[mi];
        C.inv_tauc = 1.0 / c.tauc, C.tau2 = c.tau2, C.km_rest = c.km_rest, C.tau1_rest = c.tau1_rest;
        C.a_force = pw ? c.a_scale : c.a_rest;
        C.pd0 = c.pd0, C.inv_pdt = pw ? 1.0 / c.pdt : 0.0;
        C.alpha_a = c.alpha_a, C.alpha_tau1 = c.alpha_tau1, C.alpha_km = c.alpha_km;
        C.inv_tau_fat = fat ? 1.0 / c.tau_fat : 0.0;
        C.a_fat_rest = pw ? c.a_scale : c.a_rest;  // ding2007_with_fatigue.py:198-241: A relaxes to a_scale
        C.inv_lopt = 1.0 / mu.optimal_length, C.slack = mu.tendon_slack_length;
        C.inv_cos_penn = 1.0 / std::cos(mu.pennation_angle);
        C.ar = c.ar, C.bs = c.bs, C.Is = c.Is, C.cr = c.cr;
        if (fat) {
            rest[mi * nxm + 2] = C.a_fat_rest;
            rest[mi * nxm + 3] = c.tau1_rest;
            rest[mi * nxm + 4] = c.km_rest;
        }
    }
    G.fl_on = (p->flags & CFX_MSK_FORCE_LENGTH) ? 1 : 0;
    G.fv_on = (p->flags & CFX_MSK_FORCE_VELOCITY) ? 1 : 0;
    G.fp_on = (p->flags & CFX_MSK_PASSIVE_FORCE) ? 1 : 0;

    // ---- calcium sums at every RK stage time, per muscle (ding2003.py:230-252, reference operation order)
    const double dt = p->final_time / N, hh = dt / m;
    const int Q = m * S;
    const int TM = hmed ? (T > 10 ? 20 : 10) : 1;  // Hmed: per-pulse coefficients, padded to the kernel's TMAX
    std::vector<double> cs((size_t)N * Q * nm * TM, 0.0);
    // CFX_MSK_LEGACY_CALCIUM (the revision that stored the reaching-task solutions, tests/test_reference_solution.py):
    // a window's first pulse is left out once the window holds several, and the fatigue models' r0 is Km + r0_km, so
    // cs = table(r0 = km_rest + r0_km) + (Km - km_rest) cs1 with cs1 = sum_{i >= 1} exp(-(t_i - t_{i-1}) / tau_c)
    // exp(-(t - t_i) / tau_c) over the pulses kept
    const bool legacy = (p->flags & CFX_MSK_LEGACY_CALCIUM) != 0;
    std::vector<double> cs1(legacy && fat ? (size_t)N * Q * nm : 0, 0.0);
    for (int k = 0; k < N; ++k) {
        const double* row = p->stim_rows + (size_t)k * T;
        int skip = -1;
        if (legacy) {
            int nreal = 0;
            for (int i = 0; i < T; ++i) nreal += row[i] > -1e6;
            if (nreal > 1) skip = T - nreal;
        }
        for (int mi = 0; mi < nm; ++mi) {
            const cfx_constants& c = p->muscles[mi].constants;
            const double r0 = c.km_rest + c.r0_km_relationship;
            std::vector<double> ri(T), di(T, 0.0);
            for (int i = 0; i < T; ++i) {
                ri[i] = i == 0 ? 1.0 : 1.0 + (r0 - 1.0) * std::exp(-(row[i] - row[i - 1]) / c.tauc);
                if (i > 0) di[i] = std::exp(-(row[i] - row[i - 1]) / c.tauc);
                if (i == skip) ri[i] = di[i] = 0.0;
            }
            for (int j = 0; j < m; ++j)
                for (int st = 0; st < S; ++st) {
                    double t = k * dt + j * hh;
                    if (S == 2 && st == 1) t += hh / 2;
                    if (S == 4 && (st == 1 || st == 2)) t += hh / 2;
                    if (S == 4 && st == 3) t += hh;
                    const size_t kq = (size_t)k * Q + (size_t)j * S + st;
                    if (hmed) {  // cs = sum_i coef_i lambda(I_i), formed in the kernels (hmed2018.py:97-98)
                        for (int i = 0; i < T; ++i) cs[(kq * nm + mi) * TM + i] = ri[i] * std::exp(-(t - row[i]) / c.tauc);
                        continue;
                    }
                    double sum = 0.0, sum1 = 0.0;
                    for (int i = 0; i < T; ++i) {
                        if (i == skip) continue;
                        sum = sum + ri[i] * std::exp(-(t - row[i]) / c.tauc);
                        sum1 = sum1 + di[i] * std::exp(-(t - row[i]) / c.tauc);
                    }
                    cs[kq * nm + mi] = sum;
                    if (!cs1.empty()) cs1[kq * nm + mi] = sum1;
                }
        }
    }
    MskParams& P = h->mp;
    P.B = p->batch, P.N = N, P.m = m, P.nx = nx, P.nu = nu, P.nz = nz, P.Q = Q;
    P.residual = residual ? 1 : 0, P.npw = npw, P.dt = dt, P.h = hh;
    P.T = T, P.ngk = ngk;
    P.kpb = msk_default_kpb(P.B, N);
    if (const char* e = std::getenv("CFX_MSK_KPB"))  // tuning / test override of the tangent kernel's launch shape
        P.kpb = std::max(1, std::min(N, std::atoi(e)));
    h->msk_ns = ns;

    // ---- structural Jacobian pattern (Dep pass on the host through the same RHS code)
    std::vector<uint64_t> dep(nx);
    {
        MskParams Ph = P;
        Ph.cs = cs.data();
        Ph.cs1 = cs1.empty() ? nullptr : cs1.data();
        msk_dep_pattern(nq, nm, fam, p->scheme, Ph, G, dep.data());
    }
    for (int e = 0; e < kMskMaxX * kMskMaxZ; ++e) G.jpos[e] = -1;
    int16_t pos = 0;
    for (int r = 0; r < nx; ++r) {
        for (int c = 0; c < nz; ++c)
            if (dep[r] >> c & 1ull) G.jpos[r * kMskMaxZ + c] = pos++;
        G.jneg[r] = pos++;
    }
    const int nnzk = pos;
    P.nnzk = nnzk;
    for (int k = 0; k < N; ++k)
        for (int r = 0; r < nx; ++r) {
            for (int c = 0; c < nz; ++c)
                if (dep[r] >> c & 1ull) {
                    h->jrow.push_back(k * ngk + r);
                    h->jcol.push_back(k * nz + c);
                }
            h->jrow.push_back(k * ngk + r);
            h->jcol.push_back((k + 1) * nz + r);
        }
    // sliding-window rows: +1 on the intensity control, -1 on its parameter (custom_constraints.py:102-119)
    std::vector<int32_t> sl_param, sl_joff;
    std::vector<double> imin(nm, 0.0);
    const int64_t p_off = (int64_t)N * nz + nx;
    if (ns) {
        // every muscle's window is padded with muscles_dynamics_model[0].min_pulse_intensity()
        // (custom_constraints.py:107-114; hmed2018.py:303-310), whatever the muscle's own recruitment constants
        const cfx_constants& c0 = p->muscles[0].constants;
        for (int mi = 0; mi < nm; ++mi) imin[mi] = std::atanh(-c0.cr) / c0.bs + c0.Is;
        for (int k = 0; k < N; ++k)
            for (int sidx = 0; sidx < ns; ++sidx) {
                const int mi = sidx / T, j = sidx - mi * T;
                const int rel = p->last_stim_idx[k] + 1 - T + j;
                const int pi = rel >= 0 ? p->param_offset[mi] + rel : -1;
                sl_param.push_back(pi);
                sl_joff.push_back((int32_t)h->jrow.size());
                h->jrow.push_back(k * ngk + nx + sidx);
                h->jcol.push_back(k * nz + nx + npw + sidx);
                if (pi >= 0) {
                    h->jrow.push_back(k * ngk + nx + sidx);
                    h->jcol.push_back((int32_t)(p_off + pi));
                }
            }
    }
    // marker superimposition rows after every interval's rows: nd J_g entries per row on q_node (dof order)
    const int qoff = nm * nxm;
    std::vector<MskMarker> mks(p->n_marker_pairs);
    int64_t mrow = (int64_t)N * ngk;
    for (int i = 0; i < p->n_marker_pairs; ++i) {
        const cfx_msk_marker_pair& c = p->marker_pairs[i];
        MskMarker& d = mks[i];
        std::memset(&d, 0, sizeof(d));
        d.node = c.node;
        for (int a = 0; a < 3; ++a)
            if (c.axes >> a & 1) d.axis[d.nrow++] = a;
        d.nd = std::max(c.frame[0], c.frame[1]) + 1;
        d.row0 = (int32_t)mrow;
        d.jo = (int32_t)h->jrow.size();
        for (int e = 0; e < 2; ++e) {
            d.frame[e] = c.frame[e];
            for (int a = 0; a < 3; ++a) d.pos[e][a] = c.pos[e][pf(c.frame[e])[a]];  // in the z-axis frame (above)
        }
        for (int r = 0; r < d.nrow; ++r)
            for (int j = 0; j < d.nd; ++j) {
                h->jrow.push_back((int32_t)(mrow + r));
                h->jcol.push_back(c.node * nz + qoff + j);
            }
        mrow += d.nrow;
    }
    // CFX_MSK_PULSE_WIDTH_PER_PULSE: interval k following the same pulse as interval k - 1 (same last stimulation
    // time in its window) keeps its pulse widths: rows u_k[m] - u_{k-1}[m] (+1, -1; constant J_g values), after the
    // marker rows — the decision space of per-pulse pulse-width parameters, with band-local rows
    std::vector<int32_t> ties;  // [n][2] decision indices (v[a] - v[b])
    const int64_t tie_row0 = mrow, tie_j0 = (int64_t)h->jrow.size();
    if (p->flags & CFX_MSK_PULSE_WIDTH_PER_PULSE)
        for (int k = 1; k < N; ++k)
            if (p->stim_rows[(size_t)k * T + T - 1] == p->stim_rows[(size_t)(k - 1) * T + T - 1])
                for (int mi = 0; mi < nm; ++mi) {
                    ties.push_back(k * nz + nx + mi);
                    ties.push_back((k - 1) * nz + nx + mi);
                    h->jrow.push_back((int32_t)mrow);
                    h->jcol.push_back(k * nz + nx + mi);
                    h->jrow.push_back((int32_t)mrow);
                    h->jcol.push_back((k - 1) * nz + nx + mi);
                    ++mrow;
                }
    h->n_ties = (int)(ties.size() / 2);
    h->tie_row0 = tie_row0;
    h->tie_j0 = tie_j0;
    // ---- Hessian: dense lower triangle of every interval block, then the diagonal of x_N (and, for marker pairs at
    // node N, the q_N pairs off the diagonal)
    const int nhk = nz * (nz + 1) / 2;
    P.nhk = nhk;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nz; ++i)
            for (int j = 0; j <= i; ++j) {
                h->hrow.push_back(k * nz + i);
                h->hcol.push_back(k * nz + j);
            }
    for (int r = 0; r < nx; ++r) {
        h->hrow.push_back(N * nz + r);
        h->hcol.push_back(N * nz + r);
    }
    {
        int ndN = 0;  // q_N pairs (i > j) needed by pairs at node N
        for (const MskMarker& d : mks)
            if (d.node == N) ndN = std::max(ndN, d.nd);
        std::vector<int32_t> offN((size_t)kMskMaxQ * kMskMaxQ, -1);
        for (int i = 0; i < ndN; ++i)
            for (int j = 0; j < i; ++j) {
                offN[i * kMskMaxQ + j] = (int32_t)h->hrow.size();
                h->hrow.push_back(N * nz + qoff + i);
                h->hcol.push_back(N * nz + qoff + j);
            }
        for (MskMarker& d : mks)
            for (int i = 0; i < kMskMaxQ; ++i)
                for (int j = 0; j <= i; ++j) {
                    int32_t& o = d.hoff[i * (i + 1) / 2 + j];
                    o = -1;
                    if (i >= d.nd) continue;
                    if (d.node < N)
                        o = d.node * nhk + (qoff + i) * (qoff + i + 1) / 2 + qoff + j;
                    else
                        o = i == j ? N * nhk + qoff + i : offN[i * kMskMaxQ + j];
                }
    }
    std::vector<int32_t> hdiag((size_t)(N + 1) * nz, -1);
    for (int k = 0; k < N; ++k)
        for (int e = 0; e < nz; ++e) hdiag[(size_t)k * nz + e] = k * nhk + e * (e + 1) / 2 + e;
    for (int r = 0; r < nx; ++r) hdiag[(size_t)N * nz + r] = N * nhk + r;
    // Y-space pairs (I <= J) of the stage-wise Hessian with a structurally non-zero second derivative, as
    // (I, J, lexicographic pair index) triples: a muscle's ODE reads only its own states, its own pulse width and
    // (q, qdot), and q'' is linear in the muscle forces and the residual torques, so pairs of two muscles'
    // variables vanish, and so do the residual torques' pairs with anything but q.
    std::vector<int16_t> tasks;
    {
        std::vector<int> owner(nz, -1);  // muscle index, -1 skeleton, -2 residual torque, -3 Hmed intensity
        for (int r = 0; r < nm * nxm; ++r) owner[r] = r / nxm;
        for (int i = 0; i < npw; ++i) owner[nx + i] = i;
        for (int i = npw; i < npw + nint; ++i) owner[nx + i] = -3;
        for (int i = npw + nint; i < nu; ++i) owner[nx + i] = -2;
        auto is_q = [&](int e) { return e >= nm * nxm && e < nm * nxm + nq; };
        int t = 0;
        for (int I = 0; I < nz; ++I)
            for (int J = I; J < nz; ++J, ++t) {
                const int a = owner[I], c = owner[J];
                // an intensity enters only its own lambda (linearly weighted in cn_dot): diagonal pairs only
                if ((a == -3 || c == -3) && !(a == -3 && I == J)) continue;
                if (a >= 0 && c >= 0 && a != c) continue;
                if ((a == -2 && !is_q(J)) || (c == -2 && !is_q(I))) continue;
                tasks.push_back((int16_t)I);
                tasks.push_back((int16_t)J);
                tasks.push_back((int16_t)t);
            }
        // k_msk_hpair's groups: pairs without q, with one q (swapped to come first), with two
        std::vector<int16_t> grp[3];
        for (size_t e = 0; e < tasks.size(); e += 3) {
            int16_t I = tasks[e], J = tasks[e + 1];
            const int g = (int)is_q(I) + (int)is_q(J);
            if (g == 1 && !is_q(I)) std::swap(I, J);
            grp[g].insert(grp[g].end(), {I, J, tasks[e + 2]});
        }
        tasks.clear();
        for (int g = 0; g < 3; ++g) {
            tasks.insert(tasks.end(), grp[g].begin(), grp[g].end());
            if (g < 2) h->mp.hgrp[g] = (int32_t)(grp[g].size() / 3);
        }
        h->mp.hgrp[2] = (int32_t)(grp[2].size() / 3);
    }
    h->n_htasks = (int)(tasks.size() / 3);

    // ---- objective terms
    std::vector<MskObjective> mobj;
    std::vector<double> targets;
    for (int t = 0; t < p->n_objectives; ++t) {
        const cfx_objective& o = p->objectives[t];
        const bool st = o.var_kind == CFX_VAR_STATE;
        const int lim = st ? N : N - 1;
        if ((o.var_kind != CFX_VAR_STATE && o.var_kind != CFX_VAR_CONTROL) || o.var_index < 0 ||
            o.var_index >= (st ? nx : nu) || o.node_first < 0 || o.node_last > lim || o.node_first > o.node_last ||
            (o.kind != CFX_OBJ_LAGRANGE && o.kind != CFX_OBJ_MAYER && o.kind != CFX_OBJ_MAYER_INV) ||
            (o.kind == CFX_OBJ_MAYER_INV && !st))
            return create_fail(h, CFX_EINVAL, "cfx_msk_create: invalid objective term " + std::to_string(t));
        MskObjective d{};
        d.kind = o.kind;
        d.var_kind = st ? 0 : 1;
        d.var_index = o.var_index;
        d.node_first = o.node_first;
        d.node_last = o.node_last;
        d.w_eff = o.weight * (o.kind == CFX_OBJ_LAGRANGE ? dt : 1.0);
        d.target_value = o.target_value;
        d.target_off = -1;
        if (o.target && o.kind != CFX_OBJ_MAYER_INV) {
            d.target_off = (int32_t)targets.size();
            targets.insert(targets.end(), o.target, o.target + N + 1);
        }
        mobj.push_back(d);
    }
    h->n_obj = (int)mobj.size();
    h->sz.nv = (int64_t)N * nz + nx + (ns ? p->n_params : 0);
    h->sz.ng = mrow;
    h->sz.nnz_jac = (int64_t)h->jrow.size();
    h->jconst.assign(h->jrow.size(), 0);  // the -1 on x_{k+1} of every continuity row
    for (int k = 0; k < N; ++k)
        for (int r = 0; r < nx; ++r) h->jconst[(size_t)k * nnzk + G.jneg[r]] = 1;
    for (int64_t e = 0; e < 2 * (int64_t)h->n_ties; ++e) h->jconst[(size_t)(tie_j0 + e)] = 1;
    h->sz.nnz_hess = (int64_t)h->hrow.size();
    h->sz.nx = nx;
    h->sz.nu = nu;
    h->n_mk = (int)mks.size();

    if (hipSetDevice(h->device) != hipSuccess) return create_fail(h, CFX_EHIP, "cfx_msk_create: hipSetDevice failed");
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess)
        return create_fail(h, CFX_EHIP, "cfx_msk_create: hipStreamCreate failed");
    h->stream = h->own_stream;
    auto upload = [&](void** dst, const void* src, size_t bytes) -> bool {
        if (bytes == 0) return true;
        if (hipMalloc(dst, bytes) != hipSuccess) return false;
        return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!upload((void**)&h->d_geom, &G, sizeof(G)) ||
        !upload((void**)&h->d_tab, cs.data(), cs.size() * sizeof(double)) ||
        !upload((void**)&h->d_rest, rest.data(), rest.size() * sizeof(double)) ||
        !upload((void**)&h->d_mobj, mobj.data(), mobj.size() * sizeof(MskObjective)) ||
        !upload((void**)&h->d_targets, targets.data(), targets.size() * sizeof(double)) ||
        !upload((void**)&h->d_htasks, tasks.data(), tasks.size() * sizeof(int16_t)) ||
        !upload((void**)&h->d_hdiag, hdiag.data(), hdiag.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_sl_param, sl_param.data(), sl_param.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_sl_joff, sl_joff.data(), sl_joff.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_msk_imin, imin.data(), imin.size() * sizeof(double)) ||
        !upload((void**)&h->d_mk, mks.data(), mks.size() * sizeof(MskMarker)) ||
        !upload((void**)&h->d_ties, ties.data(), ties.size() * sizeof(int32_t)) ||
        !upload((void**)&h->d_cs1, cs1.data(), cs1.size() * sizeof(double)))
        return create_fail(h, CFX_ENOMEM, "cfx_msk_create: device allocation/upload failed");
    P.cs = h->d_tab;
    P.cs1 = cs1.empty() ? nullptr : h->d_cs1;
    P.rest = h->d_rest;
    *out = h;
    return CFX_OK;
}

// per-pulse pulse-width rows v[a] - v[b] (CFX_MSK_PULSE_WIDTH_PER_PULSE): SoA, thread = (instance, row)
static __global__ void __launch_bounds__(256) k_msk_ties(int64_t B, int n, const int32_t* __restrict__ ties,
                                                         int64_t row0, int64_t j0, int keepc,
                                                         const double* __restrict__ V, double* __restrict__ G,
                                                         double* __restrict__ J) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * n) return;
    const int64_t b = item % B, t = item / B;
    if (G) G[(row0 + t) * B + b] = V[(int64_t)ties[2 * t] * B + b] - V[(int64_t)ties[2 * t + 1] * B + b];
    if (J && !keepc) {
        J[(j0 + 2 * t) * B + b] = 1.0;
        J[(j0 + 2 * t + 1) * B + b] = -1.0;
    }
}
static hipError_t launch_msk_ties(cfx_handle* h, const double* V, double* G, double* J, int keepc) {
    if (!h->n_ties || (!G && !J)) return hipSuccess;
    const int64_t items = h->mp.B * h->n_ties;
    hipLaunchKernelGGL(k_msk_ties, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, h->stream, h->mp.B, h->n_ties,
                       (const int32_t*)h->d_ties, h->tie_row0, h->tie_j0, keepc, V, G, J);
    return hipGetLastError();
}

// marker superimposition rows / their Hessian terms (k_msk_markers, one thread per instance)
static hipError_t launch_msk_markers(cfx_handle* h, const double* V, double* G, double* J, const double* LAM,
                                     double* H) {
    if (!h->n_mk) return hipSuccess;
    const MskParams& P = h->mp;
    const dim3 grid((unsigned)((P.B + 255) / 256)), blk(256);
    const int qoff = P.nx - 2 * h->msk_nq;  // q follows the muscle blocks
    switch (h->msk_nq) {
        case 1: hipLaunchKernelGGL(k_msk_markers<1>, grid, blk, 0, h->stream, P, h->d_geom, h->n_mk, h->d_mk, qoff, V, G, J, LAM, H); break;
        case 2: hipLaunchKernelGGL(k_msk_markers<2>, grid, blk, 0, h->stream, P, h->d_geom, h->n_mk, h->d_mk, qoff, V, G, J, LAM, H); break;
        case 3: hipLaunchKernelGGL(k_msk_markers<3>, grid, blk, 0, h->stream, P, h->d_geom, h->n_mk, h->d_mk, qoff, V, G, J, LAM, H); break;
        default: hipLaunchKernelGGL(k_msk_markers<4>, grid, blk, 0, h->stream, P, h->d_geom, h->n_mk, h->d_mk, qoff, V, G, J, LAM, H); break;
    }
    return hipGetLastError();
}

static int msk_eval_all(cfx_handle* h, const double* v, double* g, double* jac, double* f, double* grad,
                        uint32_t flags) {
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const int64_t B = h->prob.batch;
    const double* V = stage_in(h, S_V, v, h->sz.nv, flags, &rc);
    if (!V) return rc;
    double* G = g ? stage_out(h, S_G, g, h->sz.ng, flags, &rc) : nullptr;
    double* J = jac ? stage_out(h, S_J, jac, h->sz.nnz_jac, flags, &rc) : nullptr;
    double* F = f ? stage_out(h, S_F, f, 1, flags, &rc) : nullptr;
    double* GR = grad ? stage_out(h, S_GRAD, grad, h->sz.nv, flags, &rc) : nullptr;
    if (rc != CFX_OK) return rc;
    if (G || J) {
        MskParams P = h->mp;
        P.keepc = keep_constants(h, flags, J) ? 1 : 0;
        if (J) {  // per-stage Jacobian coefficients (and stage values) between the g + J_g launches
            const size_t nw = h->msk_stash ? msk_hess_work_host(h->msk_nq, h->msk_nm, P.nx, P.nz, P.nz * (P.nz + 1) / 2,
                                                                B, P.N, P.Q)
                                           : msk_shoot_work_host(h->msk_nq, h->msk_nm, P.nx, B, P.N, P.Q);
            P.scratch = ensure(h, h->main[S_WORK], nw, &rc);
            if (!P.scratch) return rc;
        }
        CFX_HIP(h, launch_msk_shooting(h->msk_nq, h->msk_nm, h->msk_fam, h->scheme, P, h->d_geom, V, G, J,
                                       h->msk_stash, h->stream));
        if (h->msk_ns) {
            const int64_t items = B * P.N * h->msk_ns;
            hipLaunchKernelGGL(k_msk_slide, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, h->stream, P,
                               h->msk_ns, (const int32_t*)h->d_sl_param, (const int32_t*)h->d_sl_joff,
                               (const double*)h->d_msk_imin, (int64_t)P.N * P.nz + P.nx, V, G, J);
        }
        CFX_HIP(h, launch_msk_markers(h, V, G, J, nullptr, nullptr));
        CFX_HIP(h, launch_msk_ties(h, V, G, J, P.keepc));
        if (J) {
            h->stash_valid = h->msk_stash;
            h->stash_same_point = false;
        }
    }
    if (F || GR) {
        if (GR) CFX_HIP(h, hipMemsetAsync(GR, 0, (size_t)B * h->sz.nv * sizeof(double), h->stream));
        hipLaunchKernelGGL(k_msk_objective, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, h->stream, h->mp,
                           h->n_obj, h->d_mobj, h->d_targets, V, F, GR, (const double*)nullptr, (double*)nullptr,
                           (const int32_t*)nullptr);
    }
    CFX_HIP(h, hipGetLastError());
    if (G && (rc = finish_out(h, S_G, G, g, h->sz.ng, flags)) != CFX_OK) return rc;
    if (J && (rc = finish_out(h, S_J, J, jac, h->sz.nnz_jac, flags)) != CFX_OK) return rc;
    if (F && (rc = finish_out(h, S_F, F, f, 1, flags)) != CFX_OK) return rc;
    if (GR && (rc = finish_out(h, S_GRAD, GR, grad, h->sz.nv, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

static int msk_eval_h(cfx_handle* h, const double* v, const double* obj_factor, const double* lambda, double* hess,
                      uint32_t flags) {
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const int64_t B = h->prob.batch;
    const double* V = stage_in(h, S_V, v, h->sz.nv, flags, &rc);
    if (!V) return rc;
    const double* OF = stage_in(h, S_A1, obj_factor, 1, flags, &rc);
    if (!OF) return rc;
    const double* LAM = stage_in(h, S_A2, lambda, h->sz.ng, flags, &rc);
    if (!LAM) return rc;
    double* H = stage_out(h, S_OUT, hess, h->sz.nnz_hess, flags, &rc);
    if (!H) return rc;
    // the pair kernel runs one thread per (instance, interval, stage, pair task) on a flat grid
    if ((int64_t)B * h->mp.N * h->mp.Q * h->n_htasks > (int64_t)INT32_MAX)
        return fail(h, CFX_EUNSUPPORTED, "cfx_eval_h: batch too large for one Hessian launch; split the batch");
    const size_t nw = msk_hess_work_host(h->msk_nq, h->msk_nm, h->mp.nx, h->mp.nz, h->mp.nz * (h->mp.nz + 1) / 2, B,
                                         h->mp.N, h->mp.Q);
    double* W = ensure(h, h->main[S_WORK], nw, &rc);
    if (!W) return rc;
    CFX_HIP(h, hipMemsetAsync(H, 0, (size_t)B * h->sz.nnz_hess * sizeof(double), h->stream));
    const bool reuse = h->msk_stash && h->stash_valid && h->stash_same_point;
    h->stash_valid = h->stash_same_point = false;
    CFX_HIP(h, launch_msk_hessian(h->msk_nq, h->msk_nm, h->msk_fam, h->scheme, h->mp, h->d_geom,
                                  (const int16_t*)h->d_htasks, h->n_htasks, V, LAM, H, W, reuse, h->stream));
    if (h->n_obj)
        hipLaunchKernelGGL(k_msk_objective, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, h->stream, h->mp,
                           h->n_obj, h->d_mobj, h->d_targets, V, (double*)nullptr, (double*)nullptr, OF, H,
                           (const int32_t*)h->d_hdiag);
    CFX_HIP(h, launch_msk_markers(h, V, nullptr, nullptr, LAM, H));
    CFX_HIP(h, hipGetLastError());
    if ((rc = finish_out(h, S_OUT, H, hess, h->sz.nnz_hess, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

static int msk_integrate(cfx_handle* h, const double* x0, const double* u, double* traj, uint32_t flags) {
    if (h->sz.nu > 0 && !u) return fail(h, CFX_EINVAL, "cfx_integrate: this model needs per-interval controls");
    CFX_HIP(h, hipSetDevice(h->device));
    int rc = CFX_OK;
    const int64_t nsamp = (int64_t)h->mp.N * h->mp.m + 1;
    const double* X0 = x0 ? stage_in(h, S_A1, x0, h->sz.nx, flags, &rc) : nullptr;
    if (x0 && !X0) return rc;
    const double* U = h->sz.nu ? stage_in(h, S_A2, u, (int64_t)h->mp.N * h->sz.nu, flags, &rc) : nullptr;
    if (h->sz.nu && !U) return rc;
    double* TR = stage_out(h, S_OUT, traj, nsamp * h->sz.nx, flags, &rc);
    if (!TR) return rc;
    CFX_HIP(h, launch_msk_ivp(h->msk_nq, h->msk_nm, h->msk_fam, h->scheme, h->mp, h->d_geom, X0, U, TR, h->stream));
    if ((rc = finish_out(h, S_OUT, TR, traj, nsamp * h->sz.nx, flags)) != CFX_OK) return rc;
    return sync_if_host(h, flags);
}

// ------------------------------------------------------------------------------------------------------
// cfx_gather_sum: the fixed gather table that places all-gathered value slices (include/cfx.h)
// ------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_gather_sum(int64_t batch, int64_t n_dst, const int32_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ idx, const double* __restrict__ src,
                                                    int64_t src_len, double* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = blockIdx.y;
    if (i >= n_dst || b >= batch) return;
    double acc = 0.0;
    for (int32_t s = ptr[i]; s < ptr[i + 1]; ++s) acc += src[b * src_len + idx[s]];
    dst[b * n_dst + i] = acc;
}

extern "C" int cfx_gather_sum(int64_t batch, int64_t n_dst, const int32_t* ptr, const int32_t* idx, const double* src,
                              int64_t src_len, double* dst, void* stream) {
    if (batch < 1 || n_dst < 0 || src_len < 0 || !ptr || (n_dst && (!idx || !src || !dst)) || batch > kMaxGridY) {
        g_create_error = "cfx_gather_sum: invalid arguments (batch must be in [1, 65535])";
        return CFX_EINVAL;
    }
    if (n_dst == 0) return CFX_OK;
    hipLaunchKernelGGL(k_gather_sum, dim3((unsigned)((n_dst + 255) / 256), (unsigned)batch), dim3(256), 0,
                       (hipStream_t)stream, batch, n_dst, ptr, idx, src, src_len, dst);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_gather_sum: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    return CFX_OK;
}
