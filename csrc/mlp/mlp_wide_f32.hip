// The fp32 (split3) launches of the wide layers' A-in-registers engine (forward, forward with the fused head, dW1):
// mlp_split.hip compiled a second time under CME_WIDE_F32_TU, which keeps only these three entry points, with its
// own code-generation flags (cme213_sp18_amd/_build.py UNIT_FLAGS: the machine scheduler's max-ILP strategy).
#define CME_WIDE_F32_TU 1
#include "mlp_split.hip"
