// cfx_msk_inst.h — kernel instantiation helpers shared by the cfx_inst_msk_*.hip translation units (one per
// model family pair, so the builds run in parallel).
#pragma once

#include <algorithm>
#include <cstdlib>
#include <string>

#include "cfx_msk_launch.h"

namespace cfx {


constexpr int kMskBlk = 256;

// k_msk_values' grid: (instance blocks, interval) or, below one block of instances, flat over (interval, instance)
inline dim3 msk_values_grid(const MskParams& P) {
    if (P.B < kMskBlk && P.N > 1) return dim3((unsigned)((P.B * P.N + kMskBlk - 1) / kMskBlk), 1u);
    return dim3((unsigned)((P.B + kMskBlk - 1) / kMskBlk), (unsigned)P.N);
}

template <int NQ, int NM, int FAM, int SCHEME>
void dep_t(const MskParams& P, const MskGeom& G, uint64_t* dep) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    Dep x[NX], u[NUMAX];
    for (int r = 0; r < NX; ++r) x[r].m = 1ull << r;
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
        u[i].m = dc >= 0 ? 1ull << (NX + dc) : 0ull;
    }
    msk_interval<NQ, NM, FAM, SCHEME>(P, G, 0, x, u, (const double*)nullptr);
    for (int r = 0; r < NX; ++r) dep[r] = x[r].m;
}

// Stage coefficients: one thread per stage (k_msk_stagecoef_par, the default) or per stage and half of the derivative
// directions (k_msk_stagecoef_split, CFX_MSK_STAGE=split).  cfg 5 at B = 65,536 (profiles/round5/msk_stage/): 0.563 vs
// 0.553 ms per call, g + J_g 1.405-1.426 vs 1.409-1.424 ms over three runs each — the halves' extra value work eats
// what the second wave per SIMD gains, so the simpler kernel stays the default.
inline bool msk_stage_split() {  // read at every launch, so a test can compare both kernels in one process
    const char* e = std::getenv("CFX_MSK_STAGE");
    return e && std::string(e) == "split";
}
// g + J_g: the stage coefficients and tangents fused (k_msk_stage_tangents) or the two-kernel path through the
// scratch buffer.  The fused launch holds one block of four waves per CU, so it needs many blocks: cfg 5 at B = 65,536
// 1.325-1.331 vs 1.371-1.374 ms, at 16,384 0.365 vs 0.381 ms, but at 8,192 0.206 vs 0.204 ms and at batch 1 0.078 vs
// 0.051 ms (profiles/round6/msk_fused/).  CFX_MSK_TANGENTS=fused|split forces either (read at every launch).
constexpr int64_t kMskFusedMinBlocks = 2048;  // 8 per CU
inline int msk_tangent_mode() {  // 0: by size, 1: fused, 2: two kernels
    const char* e = std::getenv("CFX_MSK_TANGENTS");
    if (e && std::string(e) == "fused") return 1;
    if (e && std::string(e) == "split") return 2;
    return 0;
}
template <int NQ, int NM, int FAM>
void msk_stagecoef(const MskParams& P, const MskGeom* G, const double* V, const double* XS, hipStream_t s) {
    const unsigned g = (unsigned)((P.B * P.N * P.Q + kMskBlk - 1) / kMskBlk);
    if (msk_stage_split())
        hipLaunchKernelGGL((k_msk_stagecoef_split<NQ, NM, FAM>), dim3(g, 2), dim3(kMskBlk), 0, s, P, G, V, XS);
    else
        hipLaunchKernelGGL((k_msk_stagecoef_par<NQ, NM, FAM>), dim3(g), dim3(kMskBlk), 0, s, P, G, V, XS);
}

// stage coefficients and tangents in one launch (k_msk_stage_tangents); keep: the Hessian that follows at this point
// reuses the coefficients, so they are stored as well
template <int NQ, int NM, int FAM, int SCHEME, int TW>
hipError_t msk_fused(const MskParams& P, const MskGeom* G, const double* V, const double* XS, double* J, int ki,
                     bool keep, hipStream_t s) {
    constexpr int NC = msk_ncoef<NQ, NM>();
    const size_t lds = (size_t)ki * P.Q * NC * TW * sizeof(double);
    static size_t raised = 65536;  // one per instantiation
    if (lds > raised) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_msk_stage_tangents<NQ, NM, FAM, SCHEME, TW>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        raised = lds;
    }
    hipLaunchKernelGGL((k_msk_stage_tangents<NQ, NM, FAM, SCHEME, TW>),
                       dim3((unsigned)((P.B + TW - 1) / TW), (unsigned)((P.N + ki - 1) / ki)), dim3(kMskFusedThreads),
                       lds, s, P, G, V, XS, J, ki, keep ? 1 : 0);
    return hipGetLastError();
}

template <int NQ, int NM, int FAM, int SCHEME>
hipError_t shoot_t(const MskParams& P, const MskGeom* G, const double* V, double* Gout, double* J, bool keep_xs,
                   hipStream_t s) {
    const unsigned gx = (unsigned)((P.B + kMskBlk - 1) / kMskBlk);
    if (!J) {  // g only: the value recursion of the g + J_g path without storing the stage inputs (CFX_MSK_G=dual: the
               // generic interval in Dual<0>, the previous kernel)
        const char* e = std::getenv("CFX_MSK_G");
        if (e && std::string(e) == "dual")
            hipLaunchKernelGGL((k_msk_shooting<NQ, NM, FAM, SCHEME, 0>), dim3(gx, (unsigned)P.N), dim3(kMskBlk), 0, s, P,
                               G, V, Gout, J);
        else
            hipLaunchKernelGGL((k_msk_values<NQ, NM, FAM, SCHEME>), msk_values_grid(P), dim3(kMskBlk), 0, s, P, G, V,
                               Gout, (double*)nullptr);
        return hipGetLastError();
    }
    // g + J_g: the value recursion (stage inputs XS), every stage's coefficients in its own thread, then one
    // thread per Jacobian column
    constexpr int NC = msk_ncoef<NQ, NM>();
    double* XS = P.scratch + P.B * P.N * P.Q * NC;
    hipLaunchKernelGGL((k_msk_values<NQ, NM, FAM, SCHEME>), msk_values_grid(P), dim3(kMskBlk), 0, s, P, G, V, Gout,
                       XS);
    const int mode = msk_tangent_mode();
    const bool fuse = P.nz <= kMskLdsCols && mode != 2;
    auto enough = [&](int tw, int ki) {
        return mode == 1 || (P.B + tw - 1) / tw * ((P.N + ki - 1) / ki) >= kMskFusedMinBlocks;
    };
    const int ki32 = fuse ? msk_fused_ki(P.N, P.Q, NC, 32) : 0;
    if (ki32 > 0 && enough(32, ki32)) return msk_fused<NQ, NM, FAM, SCHEME, 32>(P, G, V, XS, J, ki32, keep_xs, s);
    if constexpr (SCHEME == 4) {  // 16-instance blocks for long RK4 intervals (RK4 x 5); RK1 / RK2 that long run unfused
        const int ki16 = fuse && ki32 == 0 ? msk_fused_ki(P.N, P.Q, NC, 16) : 0;
        if (ki16 > 0 && enough(16, ki16))
            return msk_fused<NQ, NM, FAM, SCHEME, 16>(P, G, V, XS, J, ki16, keep_xs, s);
    }
    msk_stagecoef<NQ, NM, FAM>(P, G, V, XS, s);
    if (P.nz <= kMskLdsCols) {  // coefficients through LDS, one block per TW instances
        constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1), TW = kMskTangentInstances;  // cfx_msk_create's kpb
        const int64_t nbx = (P.B + TW - 1) / TW;
        const int kpb = std::max(1, std::min(P.N, P.kpb));  // intervals per block (cfx_msk_create)
        // two coefficient buffers when B is even (k_msk_tangents_lds): above the default 64 KiB of dynamic LDS for cfg 5
        const size_t lds = (P.B % 2 == 0 ? 2 : 1) * ST * NC * TW * sizeof(double);
        static size_t raised = 65536;  // one per instantiation
        if (lds > raised) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_msk_tangents_lds<NQ, NM, FAM, SCHEME, TW>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            raised = lds;
        }
        hipLaunchKernelGGL((k_msk_tangents_lds<NQ, NM, FAM, SCHEME, TW>), dim3((unsigned)nbx, (unsigned)((P.N + kpb - 1) / kpb)),
                           dim3(TW * P.nz), lds, s, P, G, V, J, kpb);
        return hipGetLastError();
    }
    const int flat = P.B < kMskBlk;  // (instance, column) threads: batches below one block per column
    const int64_t ranges8 = ((P.B + kMskBlk - 1) / kMskBlk + 7) / 8 * 8;  // instance ranges, padded to 8 XCDs
    const unsigned gt = flat ? (unsigned)((P.B * P.nz + kMskBlk - 1) / kMskBlk) : (unsigned)(ranges8 * P.nz);
    hipLaunchKernelGGL((k_msk_tangents<NQ, NM, FAM, SCHEME>), dim3(gt, (unsigned)P.N), dim3(kMskBlk), 0, s, P, G, V, J,
                       flat);
    return hipGetLastError();
}

template <int NQ, int NM, int FAM, int SCHEME>
hipError_t hess_t(const MskParams& P, const MskGeom* G, const int16_t* tasks, int ntasks, const double* V,
                  const double* LAM, double* H, double* work, bool reuse, hipStream_t s) {
    // work (msk_hess_work_host doubles): stage coefficients | XS | TS | MU | GQ [| HQ]
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ, NC = msk_ncoef<NQ, NM>();
    const int64_t BNQ = P.B * P.N * P.Q;
    MskParams Pw = P;
    Pw.scratch = work;
    double* XS = work + BNQ * NC;
    double* TS = XS + BNQ * NX;
    double* MU = TS + BNQ * NX * P.nz;
    double* GQ = MU + BNQ * NX;
    const int npair = P.nz * (P.nz + 1) / 2;  // GQ holds every pair; the structurally zero ones stay 0
    if (ntasks < npair) {
        const hipError_t e = hipMemsetAsync(GQ, 0, (size_t)BNQ * npair * sizeof(double), s);
        if (e != hipSuccess) return e;
    }
    const unsigned gx = (unsigned)((P.B + kMskBlk - 1) / kMskBlk);
    auto flat = [](int64_t items) { return dim3((unsigned)((items + kMskBlk - 1) / kMskBlk)); };
    const bool small = P.B <= kMskSmallBatch;
    if (!reuse) {  // stage values and coefficients (reuse: left by the g + J_g launch at this point)
        hipLaunchKernelGGL((k_msk_values<NQ, NM, FAM, SCHEME>), msk_values_grid(P), dim3(kMskBlk), 0, s, Pw, G, V,
                           (double*)nullptr, XS);
        msk_stagecoef<NQ, NM, FAM>(Pw, G, V, XS, s);
    }
    hipLaunchKernelGGL((k_msk_htan<NQ, NM, FAM, SCHEME>), flat(P.B * P.N * P.nz), dim3(kMskBlk), 0, s, Pw, G, V, TS);
    hipLaunchKernelGGL((k_msk_hadj<NQ, NM, FAM, SCHEME>), flat(P.B * P.N), dim3(kMskBlk), 0, s, Pw, G, LAM, MU);
    {  // the three task groups (k_msk_hpair), each its own instantiation and register allocation
        const int16_t* tg = tasks;
        const int n0 = P.hgrp[0], n1 = P.hgrp[1], n2 = ntasks - n0 - n1;
        if (n0 > 0)
            hipLaunchKernelGGL((k_msk_hpair<NQ, NM, FAM, 0>), flat(BNQ * n0), dim3(kMskBlk), 0, s, Pw, G, tg, n0, npair,
                               V, (const double*)XS, (const double*)MU, GQ);
        if (n1 > 0)
            hipLaunchKernelGGL((k_msk_hpair<NQ, NM, FAM, 1>), flat(BNQ * n1), dim3(kMskBlk), 0, s, Pw, G, tg + 3 * n0,
                               n1, npair, V, (const double*)XS, (const double*)MU, GQ);
        if (n2 > 0)
            hipLaunchKernelGGL((k_msk_hpair<NQ, NM, FAM, 2>), flat(BNQ * n2), dim3(kMskBlk), 0, s, Pw, G,
                               tg + 3 * (n0 + n1), n2, npair, V, (const double*)XS, (const double*)MU, GQ);
    }
    if (small) {
        double* HQ = GQ + BNQ * npair;
        const size_t lds = msk_hproj_lds(NX, P.nz);
        if (lds <= 65536 && std::getenv("CFX_MSK_HPROJ") == nullptr) {  // stages staged in LDS (CFX_MSK_HPROJ: the old kernel)
            const int64_t nkq = (int64_t)P.N * P.Q;
            hipLaunchKernelGGL((k_msk_hproj_stage_lds<NQ, NM, FAM>),
                               dim3((unsigned)((nkq + kMskHpS - 1) / kMskHpS), (unsigned)P.B), dim3(kMskHpS * kMskMaxZ), lds,
                               s, Pw, (const double*)TS, (const double*)GQ, npair, HQ);
        } else {
            hipLaunchKernelGGL((k_msk_hproj_stage<NQ, NM, FAM>), flat(BNQ * P.nz), dim3(kMskBlk), 0, s, Pw,
                               (const double*)TS, (const double*)GQ, npair, HQ);
        }
        hipLaunchKernelGGL(k_msk_hproj_sum, flat(P.B * P.N * P.nhk), dim3(kMskBlk), 0, s, Pw, (const double*)HQ, H);
    } else {
        hipLaunchKernelGGL((k_msk_hproj<NQ, NM, FAM>), flat(P.B * P.N * P.nz), dim3(kMskBlk), 0, s, Pw,
                           (const double*)TS, (const double*)GQ, npair, H);
    }
    return hipGetLastError();
}

template <int NQ, int NM, int FAM, int SCHEME>
hipError_t ivp_t(const MskParams& P, const MskGeom* G, const double* X0, const double* U, double* TR, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kMskBlk - 1) / kMskBlk));
    hipLaunchKernelGGL((k_msk_ivp<NQ, NM, FAM, SCHEME>), grid, dim3(kMskBlk), 0, s, P, G, X0, U, TR);
    return hipGetLastError();
}

// One dispatched call: op 0 = dependency pattern (host), 1 = g + J_g, 2 = Hessian, 3 = IVP, 4 = "is it compiled".
struct MskCall {
    int op, nq, nm, fam, scheme;
    const MskParams* P;
    const MskGeom* G;      // device copy (kernels) or host copy (op 0)
    uint64_t* dep;
    const double *V, *LAM, *X0, *U;
    double *Gout, *J, *H, *TR, *work;
    const int16_t* tasks;
    int ntasks;
    bool flag;  // op 1: keep the stage values; op 2: reuse the stage values and coefficients
    hipStream_t s;
    hipError_t err;
};

template <int NQ, int NM, int FAM, int SC>
bool msk_try(MskCall& c) {
    if (c.nq != NQ || c.nm != NM || c.fam != FAM || c.scheme != SC) return false;
    switch (c.op) {
        case 0: dep_t<NQ, NM, FAM, SC>(*c.P, *c.G, c.dep); break;
        case 1: c.err = shoot_t<NQ, NM, FAM, SC>(*c.P, c.G, c.V, c.Gout, c.J, c.flag, c.s); break;
        case 2: c.err = hess_t<NQ, NM, FAM, SC>(*c.P, c.G, c.tasks, c.ntasks, c.V, c.LAM, c.H, c.work, c.flag, c.s); break;
        case 3: c.err = ivp_t<NQ, NM, FAM, SC>(*c.P, c.G, c.X0, c.U, c.TR, c.s); break;
        default: break;
    }
    return true;
}

#define CFX_MSK_SCHEMES(NQ, NM, FAM) \
    msk_try<NQ, NM, FAM, 1>(c) || msk_try<NQ, NM, FAM, 2>(c) || msk_try<NQ, NM, FAM, 4>(c)

// per-shape dispatchers (cfx_inst_msk_s<nq><nm>.hip)
bool msk_dispatch_s11(MskCall& c);
bool msk_dispatch_s21(MskCall& c);
bool msk_dispatch_s22(MskCall& c);
bool msk_dispatch_s26(MskCall& c);
bool msk_dispatch_hmed(MskCall& c);

}  // namespace cfx
