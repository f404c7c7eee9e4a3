// FETCH_SIZE calibration for k_mcq's access widths (tools/fetch_calib.sh, profiles/r05s).
// MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a 16-byte-per-lane streaming read
// on gfx950, other widths are uncalibrated. k_mcq reads 12-byte (8-bit) / 24-byte (16-bit)
// window rows per lane (McqW8 / McqW16, vp9hip_kernels.hip). Each kernel here reads a 256 MiB
// buffer exactly once (every byte by one lane) in one of those widths, so FETCH_SIZE / 256 MiB
// is the factor to apply to k_mcq's counter.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef struct __attribute__((packed, aligned(1))) { uint32_t d[3]; } W12;
typedef struct __attribute__((packed, aligned(2))) { uint32_t d[6]; } W24;

template <class W>
__global__ __launch_bounds__(256) void k_read(const uint8_t *__restrict__ src, size_t n, uint32_t *__restrict__ out)
{
    const size_t per = sizeof(W), chunks = n / per;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t) 256 + threadIdx.x; i < chunks; i += (size_t) gridDim.x * 256) {
        const __attribute__((address_space(1))) W *q = (const __attribute__((address_space(1))) W *) (src + i * per);
#pragma unroll
        for (int k = 0; k < (int) (sizeof(W) / 4); k++) acc ^= q->d[k];
    }
    if (acc == 0x12345678u) out[0] = acc;          // keeps the loads
}

__global__ __launch_bounds__(256) void k_read16(const uint4 *__restrict__ src, size_t n, uint32_t *__restrict__ out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t) 256 + threadIdx.x; i < n / 16; i += (size_t) gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    const size_t n = (size_t) 256 << 20;
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, n) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, n);
    const int grid = 256 * 16;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_read16, dim3(grid), dim3(256), 0, 0, (const uint4 *) buf, n, out);
        hipLaunchKernelGGL((k_read<W12>), dim3(grid), dim3(256), 0, 0, buf, n, out);
        hipLaunchKernelGGL((k_read<W24>), dim3(grid), dim3(256), 0, 0, buf, n, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("read %zu bytes per kernel launch\n", n);
    hipFree(buf);
    hipFree(out);
    return 0;
}
