// Shared host-side plumbing of libsfmcore: error reporting, HIP checks, the
// context (device + stream + optional RCCL communicator).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/sfmcore.h"

namespace sfm {

void set_error(const char* fmt, ...);

struct SfmError {
    int code;
};

#define SFM_HIP(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            ::sfm::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,                \
                             hipGetErrorString(e_));                                     \
            throw ::sfm::SfmError{SFM_ERR_DEVICE};                                       \
        }                                                                                \
    } while (0)

#define SFM_REQUIRE(cond, code, ...)                                                     \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            ::sfm::set_error(__VA_ARGS__);                                               \
            throw ::sfm::SfmError{code};                                                 \
        }                                                                                \
    } while (0)

// Run `body` and translate exceptions into SFM_ERR_* codes (nothing throws
// across the C-ABI).
template <class F>
int guarded(F&& body) {
    try {
        return body();
    } catch (const SfmError& e) {
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return SFM_ERR_OOM;
    } catch (...) {
        set_error("unexpected C++ exception");
        return SFM_ERR_DEVICE;
    }
}

// Minimal RCCL surface, resolved at run time from the librccl.so.1 already
// loaded in the process (torch's) or from /opt/rocm.
struct Rccl;
const Rccl* rccl();  // throws SFM_ERR_COMM if unavailable
int rccl_allreduce_f64(void* comm, double* buf, size_t n, int op_max, hipStream_t s);
// out[world][n] <- every rank's in[n] (RCCL communicator only)
int rccl_allgather_f64(void* comm, const double* in, double* out, size_t n, hipStream_t s);
// All-reduce of a device buffer across the context's ranks (RCCL, or the
// host hook through pinned memory); no-op at world 1.
void ctx_allreduce(sfm_ctx* ctx, double* dev_buf, size_t n, int op_max, hipStream_t s);
int rccl_comm_init(void** comm, int world, const uint8_t* id128, int rank);
void rccl_comm_destroy(void* comm);

// Device buffer RAII.
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        reset();
        if (count == 0) return;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            set_error("hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
            throw SfmError{SFM_ERR_OOM};
        }
        n = count;
        // SFM_POISON_ALLOC=1 (tests): every fresh buffer starts as 0xFF bytes
        // (NaN doubles, -1 integers), so a read before the first write shows
        // (completed before any stream can use the buffer)
        if (poison_alloc()) {
            SFM_HIP(hipMemset(p, 0xFF, count * sizeof(T)));
            SFM_HIP(hipDeviceSynchronize());
        }
    }
    static bool poison_alloc() {
        static const bool on = std::getenv("SFM_POISON_ALLOC") != nullptr;
        return on;
    }
    void upload(const T* h, size_t count, hipStream_t s) {
        if (count) SFM_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void zero(hipStream_t s) {
        if (n) SFM_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
};

}  // namespace sfm

struct sfm_ctx {
    int device = 0;
    int rank = 0;
    int world = 1;
    hipStream_t stream = nullptr;
    void* comm = nullptr;  // ncclComm_t when world > 1 (RCCL path)
    sfm_allreduce_fn host_allreduce = nullptr;   // host-staged path instead of RCCL
    void* host_allreduce_user = nullptr;
    double* host_buf = nullptr;                  // pinned staging for host_allreduce
    size_t host_cap = 0;
    int cu_count = 0;
};
