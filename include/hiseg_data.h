/*
 * hiseg_data.h — the training data path on the GPU (src/human_edge_detection/dataset.py:85-291
 * COCOInstanceSegmentationDataset.__getitem__ without augmentation, dataset_adapter.py:7-52 collate).
 * Conventions as in hiseg.h.  Decoding (PIL / pycocotools on the host) stays outside: these entry points
 * take decoded 8-bit images and per-instance binary masks and produce, for a batch of samples,
 *   - the image resized to the training size exactly as PIL Image.resize(size, BILINEAR) (Pillow
 *     libImaging/Resample.c: separable triangle filter whose support widens with the down-scale factor,
 *     22-bit fixed-point coefficients, horizontal pass rounded to 8 bits, then the vertical pass), written
 *     as f32 CHW / 255 (dataset.py:281-284) or 8-bit HWC;
 *   - the 3-class ROI target (dataset.py:119-170 and 268-275): every instance mask nearest-resized to the
 *     image size (cv2.INTER_NEAREST), cropped to the ROI, class 1 where the target instance is set, class 2
 *     where another instance is set, 0 elsewhere, nearest-resized to the mask size -- one fused gather per
 *     output pixel (the intermediate full-size masks are never materialised).
 */
#ifndef HISEG_DATA_H_
#define HISEG_DATA_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host function (no GPU): Pillow's bilinear resampling table for one axis, in_size -> out_size over the
 * whole input (box [0, in_size]).  Fills bounds[2*out_size] = (first input index, count) and
 * kk[out_size*ksize] = 22-bit fixed-point weights; *ksize = filter taps per output (call once with kk =
 * bounds = NULL to get *ksize).  Returns HISEG_OK or an error code. */
int hiseg_pil_bilinear_table(int in_size, int out_size, int* ksize, int* bounds, int* kk);

/* Horizontal pass: src 8-bit [B][H][W][C] (C 1..4) rows y_first .. y_first+rows-1 -> tmp [B][rows][Wout][C]. */
int hiseg_pil_resample_h(const unsigned char* src, int B, int H, int W, int C, int y_first, int rows, int Wout,
                         int ksize, const int* bounds, const int* kk, unsigned char* tmp, hiseg_stream_t stream);

/* Vertical pass: tmp [B][rows][W][C] -> out [B][Hout][W][C] 8-bit (out_f32 = 0) or f32 [B][C][Hout][W] with
 * value / 255 (out_f32 = 1).  bounds are relative to the tmp rows. */
int hiseg_pil_resample_v(const unsigned char* tmp, int B, int rows, int W, int C, int Hout, int ksize,
                         const int* bounds, const int* kk, int out_f32, void* out, hiseg_stream_t stream);

/* One ROI target sample.  Instance masks of the sample: n_inst consecutive 8-bit [h0][w0] planes starting at
 * byte mask_offset of the mask buffer; target = index of the target instance among them.  (x1, y1, x2, y2):
 * the integer ROI in image-size pixels (after padding / clamping / minimum size, dataset.py:127-147);
 * (img_w, img_h): the image size the masks are resized to (dataset.py:117). */
typedef struct hiseg_roi_target_desc {
  long long mask_offset;
  int n_inst, target, h0, w0;
  int x1, y1, x2, y2;
  int img_w, img_h;
} hiseg_roi_target_desc;

/* descs: device array [B]; out int64 [B][mh][mw] class ids. */
int hiseg_roi_targets(const unsigned char* masks, const hiseg_roi_target_desc* descs, int B, int mh, int mw,
                      long long* out, hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif
