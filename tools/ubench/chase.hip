// chase.hip — dependent-load latency probe: each wave walks a random cycle of
// 16-byte records inside its own region (like one GST shard's arena), so the
// per-hop time is the round trip a GST iteration pays.  Run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 chase.hip -o chase && ./chase
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>

__global__ void chase(const uint4 *buf, uint64_t region_recs, int hops, uint64_t *out) {
    const uint4 *base = buf + (uint64_t)blockIdx.x * region_recs;
    uint32_t cur = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < hops; ++i) cur = __builtin_amdgcn_readfirstlane(base[cur].x);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = cur; }
}

__global__ void fill(uint4 *buf, uint64_t region_recs, uint32_t stride_mul) {
    // next = (i * a + c) mod region: a full-period LCG-ish permutation (region pow2)
    uint64_t n = region_recs * gridDim.y;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < region_recs; i += 256ull * gridDim.x) {
        uint64_t nx = (i * 2654435761ull + 12345ull) & (region_recs - 1);
        for (uint32_t r = 0; r < gridDim.y; ++r) buf[(uint64_t)r * region_recs + i] = make_uint4((uint32_t)nx, 0, 0, 0);
    }
    (void)n; (void)stride_mul;
}

int main() {
    const int hops = 4000;
    uint64_t regions_mb[] = {1, 4, 16, 64};
    int waves_list[] = {1, 64, 512, 2048};
    for (uint64_t rmb : regions_mb) {
        uint64_t recs = rmb * 1024 * 1024 / 16;
        for (int waves : waves_list) {
            uint64_t bytes = recs * 16 * (uint64_t)waves;
            if (bytes > (64ull << 30)) continue;
            uint4 *buf; uint64_t *out;
            if (hipMalloc(&buf, bytes) != hipSuccess) { printf("oom\n"); return 1; }
            hipMalloc(&out, 16 * waves);
            for (int r0 = 0; r0 < waves; r0 += 64) {
                int nr = waves - r0 < 64 ? waves - r0 : 64;
                hipLaunchKernelGGL(fill, dim3(1024, nr), dim3(256), 0, 0, buf + (uint64_t)r0 * recs, recs, 0);
            }
            hipDeviceSynchronize();
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(chase, dim3(waves), dim3(64), 0, 0, buf, recs, hops, out);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            std::vector<uint64_t> h(2 * waves);
            hipMemcpy(h.data(), out, 16 * waves, hipMemcpyDeviceToHost);
            double cyc = 0; for (int w = 0; w < waves; ++w) cyc += h[2 * w];
            cyc /= waves * (double)hops;
            printf("region %4llu MB waves %5d total %7.2f GB: %7.1f cyc/hop  %7.1f ns/hop (event)\n",
                   (unsigned long long)rmb, waves, bytes / 1e9, cyc, ms * 1e6 / hops);
            hipFree(buf); hipFree(out);
        }
    }
    return 0;
}
