// Weight-gradient launch arguments shared by the transposed-read kernels (train_conv.hip, wgrad_wide.hip).
#pragma once
#include "conv_common.h"

namespace hiseg {

struct WgradArgs {
  hiseg_conv2d_desc d;  // forward descriptor (input side + geometry)
  const void* dy; int dy_cs, dy_coff;
  int M;          // GEMM rows of the forward conv (output pixels; input pixels for convT)
  int Cin;        // Ca + Cb (padded)
  int Ktot;       // KH*KW*Cin
  int want_bias;
  int Cg, Kg;
  int splits, blocks_per_split;  // pixel blocks per split
  float* ws;
  int x_tile_src;  // transposed-read kernel: 0 = per-lane source over one resource spanning both; two sources
                   // too far apart for one 2^31-byte resource: 1 = one X source per K tile (the layer's tiles never
                   // mix them), 2 = one resource per source, chosen per lane (conv_wgrad_tr_kernel's XR)
};

}  // namespace hiseg
