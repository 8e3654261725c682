// Read-bandwidth probe: how fast can the chip stream a B-byte buffer that is re-read every
// launch (MALL-resident when B < ~256 MiB)?  Prints GB/s per configuration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int UNR>
__global__ __launch_bounds__(256) void rd(const f32x4 *__restrict__ p, long n, float *out) {
    f32x4 acc = {0, 0, 0, 0};
    long stride = (long)gridDim.x * blockDim.x;
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (; i + (UNR - 1) * stride < n; i += UNR * stride) {
        f32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < UNR; u++) acc += v[u];
    }
    for (; i < n; i += stride) acc += p[i];
    if (acc[0] + acc[1] + acc[2] + acc[3] == 1234.5f) out[0] = 1;
}
template <int UNR>
__global__ __launch_bounds__(256) void rd_plain(const f32x4 *__restrict__ p, long n, float *out) {
    f32x4 acc = {0, 0, 0, 0};
    long stride = (long)gridDim.x * blockDim.x;
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (; i + (UNR - 1) * stride < n; i += UNR * stride) {
        f32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = p[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNR; u++) acc += v[u];
    }
    for (; i < n; i += stride) acc += p[i];
    if (acc[0] + acc[1] + acc[2] + acc[3] == 1234.5f) out[0] = 1;
}

int main(int argc, char **argv) {
    long MB[] = {26, 52, 105, 210, 1024};
    for (long mb : MB) {
        long bytes = mb * 1000000L;
        long n = bytes / 16;
        f32x4 *p;
        float *o;
        if (hipMalloc(&p, bytes) || hipMalloc(&o, 4)) return 1;
        hipMemset(p, 0, bytes);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int cfg = 0; cfg < 6; cfg++) {
            int grid = (cfg % 3 == 0) ? 1024 : (cfg % 3 == 1) ? 2048 : 4096;
            auto launch = [&]() {
                if (cfg < 3) hipLaunchKernelGGL(rd<8>, dim3(grid), dim3(256), 0, 0, p, n, o);
                else hipLaunchKernelGGL(rd_plain<8>, dim3(grid), dim3(256), 0, 0, p, n, o);
            };
            for (int w = 0; w < 5; w++) launch();
            hipEventRecord(a);
            const int R = 50;
            for (int r = 0; r < R; r++) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%5ld MB  %s grid %5d: %7.1f us/launch  %6.2f TB/s\n", mb, cfg < 3 ? "nt   " : "plain", grid,
                   ms * 1000 / R, bytes / (ms / R * 1e-3) / 1e12);
        }
        hipFree(p);
        hipFree(o);
    }
    return 0;
}
