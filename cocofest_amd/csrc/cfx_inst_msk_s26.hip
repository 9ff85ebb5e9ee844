// cfx_inst_msk_s26.hip — musculoskeletal kernels for the arm26 (2 dofs, 6 muscles) shape, Ding2003 / Ding2007 families with and
// without fatigue, RK1 and RK4.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_s26(MskCall& c) {
    return CFX_MSK_SCHEMES(2, 6, 0) || CFX_MSK_SCHEMES(2, 6, 1) || CFX_MSK_SCHEMES(2, 6, 2) ||
           CFX_MSK_SCHEMES(2, 6, 3);
}

}  // namespace cfx
