// cfx_inst_msk_s22.hip — musculoskeletal kernels for the arm26_biceps_triceps (2 dofs, 2 muscles; BASELINE config 5) shape, Ding2003 / Ding2007 families with and
// without fatigue, RK1 and RK4.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_s22(MskCall& c) {
    return CFX_MSK_SCHEMES(2, 2, 0) || CFX_MSK_SCHEMES(2, 2, 1) || CFX_MSK_SCHEMES(2, 2, 2) ||
           CFX_MSK_SCHEMES(2, 2, 3);
}

}  // namespace cfx
