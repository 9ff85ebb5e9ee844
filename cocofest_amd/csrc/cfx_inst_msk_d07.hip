// cfx_inst_msk_d07.hip — musculoskeletal kernels for the Ding2007 (+ fatigue) muscle families.
#include "cfx_msk_inst.h"

namespace cfx {

bool msk_dispatch_d07(MskCall& c) { return CFX_MSK_SCHEMES(2, 2, 2) || CFX_MSK_SCHEMES(2, 2, 3); }

}  // namespace cfx
