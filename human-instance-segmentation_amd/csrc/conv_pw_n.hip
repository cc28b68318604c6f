// Narrow column tiles of the persistent pointwise kernel (conv_pw.hip): RB 1, 2, 4 and 8 (16..128 output
// columns) for the EfficientNet encoder's 1x1 projections and expansions, compiled as a separate object so the
// two halves build in parallel.
#define HISEG_PW_PART 2
#include "conv_pw.hip"
