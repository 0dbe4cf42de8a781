// traffic_probe.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of the O2 kernel (k_sgns_o2_ring), on known byte counts (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern before trusting an absolute").
//
// Every kernel touches a 2 GiB table (8x the 256 MiB Infinity Cache), each row / line exactly
// once per launch in a scattered order (a multiplicative bijection), so no access is served from
// L2 or the Infinity Cache.  Rows are 512 B (d = 128 fp32) and are accessed
// exactly as Row<2, true> does in come_sgns_impl.h: lane l moves elements l and l + 64, i.e. two
// dword-per-lane wave instructions of 256 contiguous bytes each.
//   k_row_read     random rows read (known read bytes = rows * 512)
//   k_row_rmw      random rows read + written with plain stores (read = write = rows * 512)
//   k_row_atomic   random rows += with no-return float atomics (rows * 512 atomic bytes)
//   k_table_read   one uint32 per lane, each from a different 64-B line (4 useful bytes per
//                  access: what one negative-table draw costs when it misses)
//   k_stream_read  16 B per lane streaming read of the whole 2 GiB table (the guide's pattern)
// Prints one JSON line with the known bytes per launch of each kernel.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o scripts/traffic_probe scripts/traffic_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

constexpr int64_t kRows = (2ll << 30) / 512;  // 4 Mi rows of 512 B = 2 GiB
constexpr int64_t kAccesses = kRows;           // every row once per launch
constexpr int64_t kLines = (2ll << 30) / 64;   // 32 Mi lines of 64 B
constexpr int64_t kTableReads = 16ll << 20;    // 4-B reads per launch, distinct lines

// i -> scattered index in [0, n), n a power of two: odd multiplier = bijection mod n
__device__ inline int64_t scatter(int64_t i, int64_t n, uint64_t salt) {
    return (int64_t)(((uint64_t)i * 0x9E3779B1ull + salt) & (uint64_t)(n - 1));
}

__global__ void __launch_bounds__(256) k_row_read(const float *__restrict__ t, float *sink) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float acc = 0.f;
    for (int64_t i = wave; i < kAccesses; i += waves) {
        const float *r = t + scatter(i, kRows, 0) * 128;
        acc += r[lane] + r[lane + 64];
    }
    if (acc == 12345.f) sink[0] = acc;  // keeps the loads; never true for this data
}

__global__ void __launch_bounds__(256) k_row_rmw(float *__restrict__ t) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < kAccesses; i += waves) {
        float *r = t + scatter(i, kRows, 12345) * 128;
        const float a = r[lane], b = r[lane + 64];
        r[lane] = a * 0.5f + 1.0f;
        r[lane + 64] = b * 0.5f + 1.0f;
    }
}

__global__ void __launch_bounds__(256) k_row_atomic(float *__restrict__ t) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < kAccesses; i += waves) {
        float *r = t + scatter(i, kRows, 777) * 128;
        atomicAdd(r + lane, 1e-3f);
        atomicAdd(r + lane + 64, 1e-3f);
    }
}

__global__ void __launch_bounds__(256) k_table_read(const uint32_t *__restrict__ table,
                                                    uint32_t *sink) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = (int64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (int64_t i = tid; i < kTableReads; i += n) acc ^= table[scatter(i, kLines, 99) * 16];
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_stream_read(const float4 *__restrict__ t, float *sink) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    for (int64_t i = tid; i < kRows * 32; i += n) {
        const float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

int main() {
    float *t = nullptr, *sink = nullptr;
    CHECK(hipMalloc(&t, kRows * 512));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(t, 0, kRows * 512));
    const uint32_t *table = (const uint32_t *)t;
    const dim3 grid(256 * 8), block(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_row_read, grid, block, 0, 0, t, sink);
        hipLaunchKernelGGL(k_row_rmw, grid, block, 0, 0, t);
        hipLaunchKernelGGL(k_row_atomic, grid, block, 0, 0, t);
        hipLaunchKernelGGL(k_table_read, grid, block, 0, 0, table, (uint32_t *)sink);
        hipLaunchKernelGGL(k_stream_read, grid, block, 0, 0, (const float4 *)t, sink);
        CHECK(hipGetLastError());
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"k_row_read\": {\"read\": %lld}, \"k_row_rmw\": {\"read\": %lld, \"write\": %lld}, "
           "\"k_row_atomic\": {\"write\": %lld}, \"k_table_read\": {\"read\": %lld, "
           "\"accesses\": %lld}, \"k_stream_read\": {\"read\": %lld}, \"launches\": 3}\n",
           (long long)(kAccesses * 512), (long long)(kAccesses * 512),
           (long long)(kAccesses * 512), (long long)(kAccesses * 512),
           (long long)(kTableReads * 4), (long long)kTableReads, (long long)(kRows * 512));
    CHECK(hipFree(t));
    CHECK(hipFree(sink));
    return 0;
}
