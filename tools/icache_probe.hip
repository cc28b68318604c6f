// Kernel time vs straight-line code size (developer tool, GPU): is a short kernel's floor its instruction fetch?
// Each kernel runs N independent v_fmac_f32 (8 B each with a literal-free encoding: 4 B) unrolled, no loop, on G
// workgroups of 256 threads, then one store per thread.  Launched `reps` times back to back (same kernel: a warm
// instruction cache if dispatch leaves it alone) and interleaved with a second kernel of the same size.
//   hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o tools/icache_probe && ./tools/icache_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int N, int TAG>
__global__ void __launch_bounds__(256) straight(float* out, float a) {
  float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1.f, x2 = x0 + 2.f, x3 = x0 + 3.f;
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    asm volatile("v_fmac_f32 %0, %4, %0\n\tv_fmac_f32 %1, %4, %1\n\tv_fmac_f32 %2, %4, %2\n\tv_fmac_f32 %3, %4, %3"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                 : "v"(a + TAG));
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3;
}

template <int N>
static void run(float* buf, int G, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms_same = 0.f, ms_alt = 0.f;
  for (int r = 0; r < 2; ++r) {   // second round timed
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((straight<N, 0>), dim3(G), dim3(256), 0, 0, buf, 1.0001f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms_same, e0, e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) {
      if (i & 1) hipLaunchKernelGGL((straight<N, 1>), dim3(G), dim3(256), 0, 0, buf, 1.0001f);
      else hipLaunchKernelGGL((straight<N, 0>), dim3(G), dim3(256), 0, 0, buf, 1.0001f);
    }
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms_alt, e0, e1);
  }
  printf("{\"instr\": %d, \"code_kb\": %.1f, \"workgroups\": %d, \"us_same\": %.2f, \"us_alternating\": %.2f}\n", N,
         N * 4 / 1024.0, G, ms_same * 1e3f / reps, ms_alt * 1e3f / reps);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  float* buf = nullptr;
  if (hipMalloc(&buf, 4096 * 256 * sizeof(float)) != hipSuccess) return 1;
  for (int G : {256, 1024}) {
    run<64>(buf, G, 200);
    run<512>(buf, G, 200);
    run<2048>(buf, G, 200);
    run<4096>(buf, G, 200);
    run<8192>(buf, G, 100);
    run<16384>(buf, G, 50);
  }
  (void)hipFree(buf);
  return 0;
}
