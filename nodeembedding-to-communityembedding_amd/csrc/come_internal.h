// Internal helpers shared by the libcome.so translation units (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/come.h"

namespace come {

// The reference's compile-time constants (pyx:18,92-93,121,134).
constexpr int kExpTableSize = 1000;
constexpr int kMaxExp = 6;
constexpr int kMaxSentenceLen = 10000;
constexpr uint64_t kLcgMul = 25214903917ULL;
constexpr uint64_t kLcgAdd = 11ULL;
constexpr uint64_t kLcgMask = (1ULL << 48) - 1;
constexpr int kMaxNegative = 20;
constexpr int kMaxDim = 512;

int set_error(int code, const char *fmt, ...);  // returns code
int hip_error(hipError_t e, const char *what);  // returns COME_E_HIP (or OK if e == success)
int ensure_init(int *device_out);               // come_init() for the current device, once
int num_cus(int device);                        // multiprocessor count (cached)
// A zeroed (on `stream`) int64 work-queue counter for one launch, or nullptr (then schedule
// statically).  Enqueues a hipMemsetAsync: capture-safe.
int64_t *launch_counter(int device, void *stream);
// Device scratch of at least `bytes` for launches on `stream` (library-owned, one buffer per
// device, stream and slot, grows on demand: the first call at a larger size allocates, so capture
// a stream only after a warm-up call of the same shape -- a growth during capture is refused).
// nullptr on failure, with the error message set: return scratch_failed() (its status code).
constexpr int kScratchGmmFlags = 0, kScratchGmmPt = 1, kScratchHotCounts = 2, kScratchHotBits = 3,
              kScratchGmmTri = 4, kScratchCommSplit = 5, kScratchRespSplit = 6,
              kScratchSlots = 7;
float *stream_scratch(int device, void *stream, int slot, size_t bytes);
int scratch_failed();
// The contended-row bitmap a Hogwild launch uses when the caller passes none (come_hot.hip):
// rows holding >= max(1, floor(share * T)) slots of `table` (share: COME_DEFAULT_HOT_SHARE for rows
// of d <= 128, COME_DEFAULT_HOT_SHARE_WIDE above) (plain uint32 or, with
// `packed`, come_pack_table's words), written into library scratch on `stream`.
int derive_hot_rows(int device, const uint32_t *table, uint64_t T, int packed, int64_t V, int d,
                    void *stream, const uint32_t **bits_out);
// One consistent snapshot of the process-wide launch options (come_set_option; mutex-guarded).
// Every entry point takes it once at its start, or uses the caller's come_launch_opts (*_ex).
come_launch_opts current_opts();

// Lemire fastmod: a % d for 32-bit a, d >= 1, from one 64-bit multiply-high.  m = 0 encodes
// "d >= 2^32" (then a % d == a for every 32-bit a).
struct FastMod {
    uint64_t m;
    uint32_t d;
};
inline FastMod make_fastmod(uint64_t T) {
    FastMod f;
    if (T >= (1ULL << 32)) {
        f.m = 0;
        f.d = 0;
    } else {
        f.d = (uint32_t)T;
        f.m = UINT64_C(0xFFFFFFFFFFFFFFFF) / f.d + 1;  // d == 1 -> m == 0 -> result 0 (correct)
    }
    return f;
}

}  // namespace come
