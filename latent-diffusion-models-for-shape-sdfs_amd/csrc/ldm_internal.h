// Internal helpers shared by the libldm_sdf.so translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>
#include <stddef.h>

#include "../../include/ldm_sdf.h"

namespace ldm {

// ---- error plumbing (ldm_last_error is thread-local, see ldm_capi.cpp) -----------------
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

#define LDM_REQUIRE(cond, code, ...)         \
    do {                                     \
        if (!(cond)) {                       \
            ::ldm::set_error(__VA_ARGS__);   \
            return (code);                   \
        }                                    \
    } while (0)

#define LDM_TRY(x)                       \
    do {                                 \
        if (int e_ = (x)) return e_;     \
    } while (0)

// hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) once per (kernel, device), thread-safe
// (a function-static flag set it once per process: a second device never got it).
template <auto Kernel>
int set_max_lds_once(int bytes, const char* what) {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static int err[kMaxDev];
    int dev = 0;
    LDM_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev, LDM_EINVAL,
                "%s: no current device", what);
    std::call_once(once[dev], [&] {
        err[dev] = (int)hipFuncSetAttribute(reinterpret_cast<const void*>(Kernel),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    });
    LDM_REQUIRE(err[dev] == 0, err[dev], "%s: hipFuncSetAttribute: %s", what,
                hipGetErrorString((hipError_t)err[dev]));
    return 0;
}

#define LDM_ALIGNED(p, a) ((((uintptr_t)(p)) & ((a) - 1)) == 0)

// Device-side invariant checks: compiled in by `make DEBUG=1` (-DLDM_DEBUG), where a failed
// check prints its location and traps the kernel (an error the host sees at the next
// synchronisation); the product build compiles them out.
#ifdef LDM_DEBUG
#define LDM_DASSERT(cond)                                                                    \
    do {                                                                                     \
        if (!(cond)) {                                                                       \
            printf("LDM_DASSERT %s:%d: %s (block %d thread %d)\n", __FILE__, __LINE__, #cond, \
                   (int)blockIdx.x, (int)threadIdx.x);                                       \
            __builtin_trap();                                                                \
        }                                                                                    \
    } while (0)
#else
#define LDM_DASSERT(cond) \
    do {                  \
    } while (0)
#endif

inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

// ---- development A/B knobs --------------------------------------------------------------
// The product library reads NO environment variable: every knob returns its default unless the
// library was built with `make DEV=1` (-DLDM_DEV_KNOBS), the build scripts/ uses for same-
// process A/B runs.  A stray variable at a caller's site can therefore never change which
// kernel runs.
#ifdef LDM_DEV_KNOBS
int dev_knob_env(const char* name, int dflt);   // capi.cpp: getenv + atoi, per call
inline int dev_knob(const char* name, int dflt) { return dev_knob_env(name, dflt); }
#else
inline int dev_knob(const char*, int dflt) { return dflt; }
#endif

// ---- fragment types ---------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Decoder kernel geometry.
constexpr int kHidden = 512;
constexpr int kTilePoints = 128;   // points per workgroup tile (4 point chunks of 32)

// feature-split decoder (decoder_fs.hip)
size_t decoder_fs_aux_bytes(int B);
int decoder_fs_n_stages(int skip_width);
int decoder_fs_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                   int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                   hipStream_t s, int num_cus);

// matrix-core path of ldm_linear (linear_mfma.hip)
int linear_mfma(const ldm_linear_args_t& a, hipStream_t s);
int64_t linear_mfma_ws_floats(const ldm_linear_args_t& a);   // split-K workspace

}  // namespace ldm
