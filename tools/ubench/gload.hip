// Microbenchmark: scattered vector loads per lane inside a small (cache-resident) buffer --
// the address rate that bounds k_gather (one unaligned 16-byte load per span piece).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/gload.hip -o /tmp/gload && /tmp/gload
// Prints, per access kind, lane-loads per second over the whole chip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
#define GAS __attribute__((address_space(1)))

template <int KIND>
__global__ void __launch_bounds__(256) k_load(const unsigned char *buf, unsigned mask, unsigned iters, unsigned *out) {
    unsigned x = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + 12345u;
    unsigned acc = 0;
    const GAS unsigned char *b = (const GAS unsigned char *)buf;
    for (unsigned i = 0; i < iters; i += 8) {
        unsigned off[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x = x * 1664525u + 1013904223u;
            off[k] = (x >> 4) & mask;
            if (KIND == 0) off[k] &= ~15u;  // aligned 16 B
            if (KIND == 2) off[k] &= ~3u;   // aligned 4 B
            if (KIND == 3) off[k] &= ~63u;  // one lane per 64-byte line, aligned 16 B
        }
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (KIND == 2) v[k] = u32x4{*(const GAS unsigned *)(b + off[k]), 0u, 0u, 0u};
            else v[k] = *(const GAS u32x4_u *)(b + off[k]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t maxb = 256u << 20;
    unsigned char *buf;
    unsigned *out;
    CK(hipMalloc(&buf, maxb + 64));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 7, maxb + 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned blocks = 256 * 8, iters = 512;
    const char *names[] = {"16B aligned", "16B unaligned", "4B aligned", "16B, one per 64B line"};
    // buffer sizes: L2-resident, a config-3 chunk's compressed bytes (~6.4 MB), past the MALL
    for (size_t bytes : {size_t(1) << 20, size_t(8) << 20, size_t(256) << 20}) {
    printf("buffer %zu MB\n", bytes >> 20);
    for (int kind = 0; kind < 4; ++kind) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(a));
            switch (kind) {
            case 0: k_load<0><<<blocks, 256>>>(buf, (unsigned)bytes - 1, iters, out); break;
            case 1: k_load<1><<<blocks, 256>>>(buf, (unsigned)bytes - 1, iters, out); break;
            case 2: k_load<2><<<blocks, 256>>>(buf, (unsigned)bytes - 1, iters, out); break;
            default: k_load<3><<<blocks, 256>>>(buf, (unsigned)bytes - 1, iters, out); break;
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double loads = (double)blocks * 256 * iters;
            if (rep == 2) printf("%-24s %8.3f ms  %7.1f G lane-loads/s  (%.0f per CU per us)\n", names[kind], ms,
                                 loads / ms / 1e6, loads / ms / 1e3 / 256 / 1e3);
        }
    }
    }
    return 0;
}
