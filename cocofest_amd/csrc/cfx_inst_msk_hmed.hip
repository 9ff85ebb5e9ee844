// cfx_inst_msk_hmed.hip — musculoskeletal kernels for Hmed2018 muscles (pulse intensities as controls, kernel
// families 4 / 5 for truncation <= 10, 6 / 7 for <= 20): the arm26_biceps_triceps (2 dofs, 2 muscles; the
// reference's tests/shard2/test_fes_dynamics.py:104-183 shape) and arm26_biceps_1dof (1, 1) shapes, RK1 / RK2 / RK4.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_hmed(MskCall& c) {
    return CFX_MSK_SCHEMES(2, 2, 4) || CFX_MSK_SCHEMES(2, 2, 5) || CFX_MSK_SCHEMES(2, 2, 6) ||
           CFX_MSK_SCHEMES(2, 2, 7) || CFX_MSK_SCHEMES(1, 1, 4) || CFX_MSK_SCHEMES(1, 1, 5) ||
           CFX_MSK_SCHEMES(1, 1, 6) || CFX_MSK_SCHEMES(1, 1, 7);
}

}  // namespace cfx
