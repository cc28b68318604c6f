// Diagnostic allocator (developer tool, not part of the library): every device allocation is a fresh hipMalloc
// filled with one byte pattern (HISEG_FILL_BYTE, default 0xFF: NaN in bf16 / f32), freed with hipFree.  Loaded
// into PyTorch through torch.cuda.memory.CUDAPluggableAllocator by tools/fill_probe.py: a kernel that reads
// memory nobody wrote then meets the pattern instead of whatever the caching allocator last held there.
#include <hip/hip_runtime.h>
#include <sys/types.h>
#include <cstdlib>

extern "C" void* fill_malloc(ssize_t size, int device, hipStream_t stream) {
  static const int byte = getenv("HISEG_FILL_BYTE") ? (int)strtol(getenv("HISEG_FILL_BYTE"), nullptr, 0) : 0xFF;
  void* p = nullptr;
  (void)device;
  if (hipMalloc(&p, size < 512 ? 512 : size) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, byte, size < 512 ? 512 : size, stream) != hipSuccess) return nullptr;
  return p;
}

extern "C" void fill_free(void* p, ssize_t size, int device, hipStream_t stream) {
  (void)size; (void)device;
  (void)hipStreamSynchronize(stream);
  (void)hipFree(p);
}
