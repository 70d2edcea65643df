// stores.hip — cost of the GST kernel's store pattern: a dependent load chain with
// K 16-byte stores per hop issued (a) by all 64 lanes to the same address, (b) by
// lane 0 only, (c) none.  Run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

template <int MODE, int K>
__global__ void __launch_bounds__(64) chase(const uint4 *buf_, uint4 *sink_, uint64_t region, int hops, uint64_t *out) {
    const G u32x4 *base = (const G u32x4 *)buf_ + (uint64_t)blockIdx.x * region;
    G u32x4 *sink = (G u32x4 *)sink_ + (uint64_t)blockIdx.x * region;
    uint32_t cur = 0, w = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < hops; ++i) {
        cur = __builtin_amdgcn_readfirstlane(base[cur].x);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t a = (cur * 7 + k * 977 + w) & (uint32_t)(region - 1);
            if (MODE == 0 || (MODE == 1 && threadIdx.x == 0)) sink[a] = u32x4{cur, (uint32_t)k, w, 1u};
            ++w;
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = cur; }
}

__global__ void fill(uint4 *buf, uint64_t region, int nreg) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < region; i += 256ull * gridDim.x) {
        uint64_t nx = (i * 2654435761ull + 12345ull) & (region - 1);
        for (int r = 0; r < nreg; ++r) buf[(uint64_t)r * region + i] = make_uint4((uint32_t)nx, 0, 0, 0);
    }
}

template <int MODE, int K>
void run(const char *name, uint4 *buf, uint4 *sink, uint64_t region, int waves, uint64_t *out) {
    const int hops = 4000;
    hipLaunchKernelGGL((chase<MODE, K>), dim3(waves), dim3(64), 0, 0, buf, sink, region, hops, out);
    hipDeviceSynchronize();
    std::vector<uint64_t> h(2 * waves);
    hipMemcpy(h.data(), out, 16 * waves, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int w = 0; w < waves; ++w) cyc += h[2 * w];
    printf("%-10s K=%d waves %4d: %7.1f cyc/hop\n", name, K, waves, cyc / (waves * (double)hops));
}

int main() {
    uint64_t region = 1u << 20;  // 16 MB of records per wave
    for (int waves : {128, 512, 2048}) {
        uint4 *buf, *sink; uint64_t *out;
        hipMalloc(&buf, region * 16 * waves);
        hipMalloc(&sink, region * 16 * waves);
        hipMalloc(&out, 16 * waves);
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, buf, region, waves);
        hipDeviceSynchronize();
        run<2, 6>("none", buf, sink, region, waves, out);
        run<0, 6>("all-lanes", buf, sink, region, waves, out);
        run<1, 6>("lane0", buf, sink, region, waves, out);
        run<0, 2>("all-lanes", buf, sink, region, waves, out);
        run<1, 2>("lane0", buf, sink, region, waves, out);
        hipFree(buf); hipFree(sink); hipFree(out);
    }
    return 0;
}
