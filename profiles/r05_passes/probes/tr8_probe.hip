// Probe of ds_read_b64_tr_b8 lane semantics on gfx950: LDS byte i holds (i & 0xff) ^ (i >> 8)*0x35;
// each lane supplies address 8*lane (lanes read the linear 512-B image in 8-B pieces) and we print
// which LDS byte index ended up in each (lane, byte) slot.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(int* out, int mode, int hi) {
  __shared__ unsigned char lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (unsigned char)(hi ? (i >> 8) : (i & 0xff));
  __syncthreads();
  const int lane = threadIdx.x;
  // mode 0: lane address = 8*lane (bytes 0..511). mode 1: = 128*lane (stride rows) within 8 KB? cap at 4 KB
  int addr = mode == 0 ? 8 * lane : (lane % 32) * 128 + (lane / 32) * 8;
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + addr));
  out[lane * 2] = r[0];
  out[lane * 2 + 1] = r[1];
}
int main() {
  int* d; (void)hipMalloc(&d, 512);
  int h[128], h2[128];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode, 0);
    (void)hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode, 1);
    (void)hipMemcpy(h2, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d (lane: 8 bytes as source byte indices)\n", mode);
    for (int l = 0; l < 64; ++l) {
      unsigned char* b = (unsigned char*)&h[l * 2];
      unsigned char* b2 = (unsigned char*)&h2[l * 2];
      printf("L%02d:", l);
      for (int j = 0; j < 8; ++j) printf(" %4d", b[j] + 256 * b2[j]);
      printf(l % 2 ? "\n" : "   |");
    }
  }
  return 0;
}
