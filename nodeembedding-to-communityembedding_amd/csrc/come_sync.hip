// come_sync.hip -- fused elementwise passes of the overlapped delta all-reduce
// (come_amd.distributed.DeltaAllReduce).  Pure HBM streams, float4 per lane,
// grid-stride over n floats.
//   begin:  D = W - S;  Down = D                        (2 reads, 2 writes per element)
//   end:    S += Dsum;  W += Dsum - Down                (4 reads, 2 writes per element)
// Row-sparse forms (SparseDeltaAllReduce): only the rows some rank changed are exchanged.
//   flags:   flag[r] = 1 iff row r of W differs bitwise from row r of S     (2 reads / element)
//   gather:  D[i] = W[idx[i]] - S[idx[i]];  Down = D                     (on the n listed rows)
//   scatter: S[idx[i]] += Dsum[i];  W[idx[i]] += Dsum[i] - Down[i]
// A row no rank changed has W == S bitwise on every rank, so its dense delta is exactly +0 and
// skipping it leaves every table bit-identical to the dense exchange.
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

__global__ void __launch_bounds__(256) k_delta_flags(const uint4 *__restrict__ W,
                                                     const uint4 *__restrict__ S, int64_t rows,
                                                     int d4, uint8_t *__restrict__ flags) {
    const int64_t n = rows * d4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256) {
        const uint4 w = W[i], s = S[i];
        if (w.x != s.x || w.y != s.y || w.z != s.z || w.w != s.w) flags[i / d4] = 1;
    }
}

__global__ void __launch_bounds__(256) k_delta_gather(const float4 *__restrict__ W,
                                                      const float4 *__restrict__ S,
                                                      const int64_t *__restrict__ idx, int64_t n,
                                                      int d4, float4 *__restrict__ D,
                                                      float4 *__restrict__ Down) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * d4;
         i += (int64_t)gridDim.x * 256) {
        const int64_t src = idx[i / d4] * d4 + i % d4;
        const float4 w = W[src], s = S[src];
        const float4 v = make_float4(w.x - s.x, w.y - s.y, w.z - s.z, w.w - s.w);
        D[i] = v;
        Down[i] = v;
    }
}

__global__ void __launch_bounds__(256) k_delta_scatter(float4 *__restrict__ W,
                                                       float4 *__restrict__ S,
                                                       const int64_t *__restrict__ idx, int64_t n,
                                                       int d4, const float4 *__restrict__ Dsum,
                                                       const float4 *__restrict__ Down) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * d4;
         i += (int64_t)gridDim.x * 256) {
        const int64_t dst = idx[i / d4] * d4 + i % d4;
        const float4 ds = Dsum[i], dn = Down[i];
        float4 s = S[dst], w = W[dst];
        s.x += ds.x, s.y += ds.y, s.z += ds.z, s.w += ds.w;
        w.x += ds.x - dn.x, w.y += ds.y - dn.y, w.z += ds.z - dn.z, w.w += ds.w - dn.w;
        S[dst] = s;
        W[dst] = w;
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

static int check_rows(const void *a, const void *b, int64_t rows, int d, const char *what) {
    if (rows < 0 || d < 4 || d % 4)
        return set_error(COME_E_INVALID, "%s: need rows >= 0 and d % 4 == 0 (got d=%d)", what, d);
    if (!ok16(a) || !ok16(b)) return set_error(COME_E_INVALID, "%s: tables must be 16-B aligned",
                                               what);
    return COME_OK;
}

extern "C" int come_delta_flags(const float *W, const float *S, int64_t rows, int d,
                                uint8_t *flags, void *stream) {
    int rc = check_rows(W, S, rows, d, "delta_flags");
    if (rc) return rc;
    if (rows == 0) return COME_OK;
    if (!flags) return set_error(COME_E_INVALID, "delta_flags: null flags");
    int dev = 0;
    rc = ensure_init(&dev);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(flags, 0, (size_t)rows, (hipStream_t)stream);
    if (e != hipSuccess) return hip_error(e, "hipMemsetAsync(flags)");
    hipLaunchKernelGGL(k_delta_flags, dim3(grid_for(rows * (d / 4), dev)), dim3(256), 0,
                       (hipStream_t)stream, (const uint4 *)W, (const uint4 *)S, rows, d / 4,
                       flags);
    return hip_error(hipGetLastError(), "k_delta_flags launch");
}

extern "C" int come_delta_gather(const float *W, const float *S, const int64_t *idx, int64_t n,
                                 int d, float *D, float *Down, void *stream) {
    int rc = check_rows(W, S, n, d, "delta_gather");
    if (rc) return rc;
    if (n == 0) return COME_OK;
    if (!idx || !ok16(D) || !ok16(Down))
        return set_error(COME_E_INVALID, "delta_gather: null index or unaligned buffers");
    int dev = 0;
    rc = ensure_init(&dev);
    if (rc) return rc;
    hipLaunchKernelGGL(k_delta_gather, dim3(grid_for(n * (d / 4), dev)), dim3(256), 0,
                       (hipStream_t)stream, (const float4 *)W, (const float4 *)S, idx, n, d / 4,
                       (float4 *)D, (float4 *)Down);
    return hip_error(hipGetLastError(), "k_delta_gather launch");
}

extern "C" int come_delta_scatter(float *W, float *S, const int64_t *idx, int64_t n, int d,
                                  const float *Dsum, const float *Down, void *stream) {
    int rc = check_rows(W, S, n, d, "delta_scatter");
    if (rc) return rc;
    if (n == 0) return COME_OK;
    if (!idx || !ok16(Dsum) || !ok16(Down))
        return set_error(COME_E_INVALID, "delta_scatter: null index or unaligned buffers");
    int dev = 0;
    rc = ensure_init(&dev);
    if (rc) return rc;
    hipLaunchKernelGGL(k_delta_scatter, dim3(grid_for(n * (d / 4), dev)), dim3(256), 0,
                       (hipStream_t)stream, (float4 *)W, (float4 *)S, idx, n, d / 4,
                       (const float4 *)Dsum, (const float4 *)Down);
    return hip_error(hipGetLastError(), "k_delta_scatter launch");
}
