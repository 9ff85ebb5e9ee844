// cfx_inst_msk_s21.hip — musculoskeletal kernels for the arm26_biceps (2 dofs, 1 muscle) shape, Ding2003 / Ding2007 families with and
// without fatigue, RK1 and RK4.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_s21(MskCall& c) {
    return CFX_MSK_SCHEMES(2, 1, 0) || CFX_MSK_SCHEMES(2, 1, 1) || CFX_MSK_SCHEMES(2, 1, 2) ||
           CFX_MSK_SCHEMES(2, 1, 3);
}

}  // namespace cfx
