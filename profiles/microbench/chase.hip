// chase.hip -- dependent-load latency on gfx950 (one lane, one wave): a random cyclic permutation
// over N 128-byte records is chased for K steps after a warm-up pass; prints ns per load for
// working sets from L2-resident to HBM-sized.  Used to price a Mode X traversal step.
//   hipcc --offload-arch=gfx950 -O3 chase.hip -o chase && ./chase
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

__global__ void chase(const int* next, int start, int steps, long long* out_cycles, int* out_end) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int p = start;
    for (int i = 0; i < steps; ++i) p = next[p * 32];   // warm
    const long long t0 = wall_clock64();
    for (int i = 0; i < steps; ++i) p = next[p * 32];
    const long long t1 = wall_clock64();
    out_cycles[0] = t1 - t0;
    out_end[0] = p;
}

int main() {
    const size_t sizes_kb[] = {64, 1024, 3072, 8192, 16384, 65536, 262144, 1048576};
    long long* dc; int* de;
    hipMalloc(&dc, sizeof(long long)); hipMalloc(&de, sizeof(int));
    for (size_t kb : sizes_kb) {
        const int n = (int)(kb * 1024 / 128);
        std::vector<int> perm(n), next((size_t)n * 32, 0);
        for (int i = 0; i < n; ++i) perm[i] = i;
        std::mt19937 rng(7);
        std::shuffle(perm.begin(), perm.end(), rng);
        for (int i = 0; i < n; ++i) next[(size_t)perm[i] * 32] = perm[(i + 1) % n];
        int* d; hipMalloc(&d, next.size() * sizeof(int));
        hipMemcpy(d, next.data(), next.size() * sizeof(int), hipMemcpyHostToDevice);
        const int steps = std::min(n, 20000);
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, perm[0], steps, dc, de);
        long long cyc; hipMemcpy(&cyc, dc, sizeof cyc, hipMemcpyDeviceToHost);
        std::printf("{\"working_set_kb\": %zu, \"ns_per_dependent_load\": %.1f}\n", kb, cyc * 10.0 / steps);   // 100 MHz clock
        hipFree(d);
    }
    return 0;
}
