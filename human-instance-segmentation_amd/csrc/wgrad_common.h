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
  int x_tile_src;  // transposed-read kernel: 1 = one X source per K tile (two sources too far apart for one
                   // buffer resource; the layer's tiles never mix them), 0 = per-lane source over one resource
};

}  // namespace hiseg
