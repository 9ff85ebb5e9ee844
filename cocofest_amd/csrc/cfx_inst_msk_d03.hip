// cfx_inst_msk_d03.hip — musculoskeletal kernels for the Ding2003 (+ fatigue) muscle families.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_d03(MskCall& c) { return CFX_MSK_SCHEMES(2, 2, 0) || CFX_MSK_SCHEMES(2, 2, 1); }

}  // namespace cfx
