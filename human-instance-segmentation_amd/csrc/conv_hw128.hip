// BCO-128 configurations of the halo-tiled wide convolution (conv_hw.hip), compiled with the MFMA accumulators
// in VGPRs (the Makefile's default flags) so that every configuration runs two waves per SIMD.
#define HISEG_HW_PART 2
#include "conv_hw.hip"
