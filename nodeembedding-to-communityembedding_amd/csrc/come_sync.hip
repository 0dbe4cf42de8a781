// come_sync.hip -- fused elementwise passes of the overlapped delta all-reduce
// (come_amd.distributed.DeltaAllReduce).  Pure HBM streams, float4 per lane,
// grid-stride over n floats.
//   begin:  D = W - S;  Down = D                        (2 reads, 2 writes per element)
//   end:    S += Dsum;  W += Dsum - Down                (4 reads, 2 writes per element)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "come_internal.h"

namespace come {

__global__ void __launch_bounds__(256) k_delta_begin(const float4 *__restrict__ W,
                                                     const float4 *__restrict__ S,
                                                     float4 *__restrict__ D,
                                                     float4 *__restrict__ Down, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * 256) {
        const float4 w = W[i], s = S[i];
        const float4 d = make_float4(w.x - s.x, w.y - s.y, w.z - s.z, w.w - s.w);
        D[i] = d;
        Down[i] = d;
    }
}

__global__ void __launch_bounds__(256) k_delta_end(float4 *__restrict__ W, float4 *__restrict__ S,
                                                   const float4 *__restrict__ Dsum,
                                                   const float4 *__restrict__ Down, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * 256) {
        const float4 ds = Dsum[i], dn = Down[i];
        float4 s = S[i], w = W[i];
        s.x += ds.x, s.y += ds.y, s.z += ds.z, s.w += ds.w;
        w.x += ds.x - dn.x, w.y += ds.y - dn.y, w.z += ds.z - dn.z, w.w += ds.w - dn.w;
        S[i] = s;
        W[i] = w;
    }
}

static int grid_for(int64_t n4, int dev) {
    int64_t b = (n4 + 255) / 256;
    const int64_t cap = (int64_t)num_cus(dev) * 8;
    return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

static bool ok16(const void *p) { return ((uintptr_t)p % 16) == 0; }

}  // namespace come

using namespace come;

extern "C" int come_delta_begin(const float *W, const float *S, float *D, float *Down, int64_t n,
                                void *stream) {
    if (n < 0 || n % 4) return set_error(COME_E_INVALID, "delta_begin: n must be >= 0, n % 4 == 0");
    if (n == 0) return COME_OK;
    if (!ok16(W) || !ok16(S) || !ok16(D) || !ok16(Down))
        return set_error(COME_E_INVALID, "delta_begin: buffers must be 16-byte aligned");
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    hipLaunchKernelGGL(k_delta_begin, dim3(grid_for(n / 4, dev)), dim3(256), 0,
                       (hipStream_t)stream, (const float4 *)W, (const float4 *)S, (float4 *)D,
                       (float4 *)Down, n / 4);
    return hip_error(hipGetLastError(), "k_delta_begin launch");
}

extern "C" int come_delta_end(float *W, float *S, const float *Dsum, const float *Down, int64_t n,
                              void *stream) {
    if (n < 0 || n % 4) return set_error(COME_E_INVALID, "delta_end: n must be >= 0, n % 4 == 0");
    if (n == 0) return COME_OK;
    if (!ok16(W) || !ok16(S) || !ok16(Dsum) || !ok16(Down))
        return set_error(COME_E_INVALID, "delta_end: buffers must be 16-byte aligned");
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    hipLaunchKernelGGL(k_delta_end, dim3(grid_for(n / 4, dev)), dim3(256), 0, (hipStream_t)stream,
                       (float4 *)W, (float4 *)S, (const float4 *)Dsum, (const float4 *)Down,
                       n / 4);
    return hip_error(hipGetLastError(), "k_delta_end launch");
}
