// cfx_inst_msk.hip — dispatch of the musculoskeletal kernels over the shapes compiled in by the
// cfx_inst_msk_s<nq><nm>.hip units (cfx_msk_inst.h).
//
// Shapes (n_dof, n_muscles): the reference's arm26 models (examples/msk_models/*.bioMod) reduced to serial
// chains — arm26_biceps_1dof (1, 1), arm26_biceps (2, 1), arm26_biceps_triceps (2, 2, BASELINE config 5),
// arm26 (2, 6).  Families: Ding2003 / Ding2007, with and without
// fatigue; schemes RK1 and RK4 (OcpFesMsk's default is RK4 x 1, fes_ocp_dynamics.py:168).
#include "cfx_msk_inst.h"

namespace cfx {

namespace {

bool dispatch(MskCall& c) {
    return msk_dispatch_s22(c) || msk_dispatch_s21(c) || msk_dispatch_s11(c) || msk_dispatch_s26(c) ||
           msk_dispatch_hmed(c);
}

MskCall make(int op, int nq, int nm, int fam, int scheme) {
    MskCall c{};
    c.op = op, c.nq = nq, c.nm = nm, c.fam = fam, c.scheme = scheme;
    c.err = hipSuccess;
    return c;
}

}  // namespace

bool msk_supported(int nq, int nm, int fam, int scheme) {
    MskCall c = make(4, nq, nm, fam, scheme);
    return dispatch(c);
}

void msk_dep_pattern(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom& G, uint64_t* dep) {
    MskCall c = make(0, nq, nm, fam, scheme);
    c.P = &P, c.G = &G, c.dep = dep;
    dispatch(c);
}

hipError_t launch_msk_shooting(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                               const double* V, double* Gout, double* J, bool keep_xs, hipStream_t s) {
    MskCall c = make(1, nq, nm, fam, scheme);
    c.P = &P, c.G = G, c.V = V, c.Gout = Gout, c.J = J, c.flag = keep_xs, c.s = s;
    return dispatch(c) ? c.err : hipErrorInvalidValue;
}

hipError_t launch_msk_hessian(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                              const int16_t* tasks, int ntasks, const double* V, const double* LAM, double* H,
                              double* work, bool reuse, hipStream_t s) {
    MskCall c = make(2, nq, nm, fam, scheme);
    c.P = &P, c.G = G, c.tasks = tasks, c.ntasks = ntasks, c.V = V, c.LAM = LAM, c.H = H, c.work = work;
    c.flag = reuse, c.s = s;
    return dispatch(c) ? c.err : hipErrorInvalidValue;
}

hipError_t launch_msk_ivp(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                          const double* X0, const double* U, double* TR, hipStream_t s) {
    MskCall c = make(3, nq, nm, fam, scheme);
    c.P = &P, c.G = G, c.X0 = X0, c.U = U, c.TR = TR, c.s = s;
    return dispatch(c) ? c.err : hipErrorInvalidValue;
}

}  // namespace cfx
