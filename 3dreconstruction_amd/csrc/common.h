// Shared host-side plumbing of libsfmcore: error reporting, HIP checks, the
// context (device + stream + optional RCCL communicator).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <new>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/sfmcore.h"

struct sfm_ctx;

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

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for the current device,
// once per (device, kernel) and raised only when a launch needs more:
// attributes are per device, and contexts of one process may drive several
// devices from several threads (ctx.cpp, under a mutex).
void set_dyn_lds(const void* kernel, size_t bytes);
// compute units of the current device (cached per device)
int device_cu_count();

// Device memory cache (ctx.cpp).  A block freed while a context is bound to
// the calling thread (CtxScope) is kept for later allocations under the same
// context stream instead of going back through hipFree, which synchronises
// the whole device and dominated small solves (a fresh plan per
// BundleAdjuster call).  Reuse is stream-ordered, so no extra synchronisation
// is needed; without a bound context blocks go straight to hipMalloc/hipFree.
void* dev_alloc(size_t bytes);   // throws SFM_ERR_OOM
void dev_free(void* p);
void dev_cache_release(hipStream_t s);   // hipFree every cached block of s
// Page-locked, device-mapped host memory, cached the same way.
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);
// Host staging memory for uploads: page-locked and cached like the above
// while a context is bound (no page faults on reuse, DMA uploads), plain
// malloc otherwise.  host_free takes either kind.
void* host_alloc(size_t bytes);
void host_free(void* p);

// std::vector allocator over host_alloc that default-initialises (resize
// does not zero-fill what the planner overwrites anyway)
template <class T>
struct HostAlloc {
    using value_type = T;
    HostAlloc() = default;
    template <class U>
    HostAlloc(const HostAlloc<U>&) noexcept {}
    T* allocate(size_t n) { return static_cast<T*>(host_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t) noexcept { host_free(p); }
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const HostAlloc<U>&) const noexcept { return true; }
    template <class U>
    bool operator!=(const HostAlloc<U>&) const noexcept { return false; }
};
template <class T>
using HostVec = std::vector<T, HostAlloc<T>>;

// Binds a context to the calling thread for the duration of an API call:
// its device, and its stream as the key of the device memory cache.
struct CtxScope {
    hipStream_t prev;
    explicit CtxScope(const sfm_ctx* c);
    ~CtxScope();
};

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
        if (p) dev_free(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        reset();
        if (count == 0) return;
        p = static_cast<T*>(dev_alloc(count * sizeof(T)));
        n = count;
        // SFM_POISON_ALLOC=1 (tests): every fresh buffer starts as 0xFF bytes
        // (NaN doubles, -1 integers), so a read before the first write shows
        // (completed before any stream can use the buffer)
        if (poison_alloc()) {
            SFM_HIP(hipDeviceSynchronize());   // a cached block's last user may still run
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

// SFM_TIMING=1 (diagnostic): host wall time per phase of a call, printed to
// stderr as "[timing] <what>: a 1.2 ms, b 3.4 ms".
struct PhaseTimer {
    static bool on() {
        static const bool v = std::getenv("SFM_TIMING") != nullptr;
        return v;
    }
    const char* what;
    double t_last;
    std::string line;
    explicit PhaseTimer(const char* w) : what(w), t_last(now()) {}
    static double now() {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
    }
    void mark(const char* phase) {
        if (!on()) return;
        const double t = now();
        char b[96];
        std::snprintf(b, sizeof b, "%s%s %.2f ms", line.empty() ? "" : ", ", phase, t - t_last);
        line += b;
        t_last = t;
    }
    ~PhaseTimer() {
        if (on() && !line.empty()) std::fprintf(stderr, "[timing] %s: %s\n", what, line.c_str());
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
    bool no_exchange = false;                    // SFM_CTX_DIAG_NO_EXCHANGE (per-rank timing only)
    bool fail_solve_wait = false;                // SFM_CTX_DIAG_FAIL_SOLVE_WAIT (error-path tests)
    bool time_kernels = false;                   // SFM_CTX_TIME_KERNELS (sfm_ctx_last_kernel_ms)
    int32_t flags = 0;                           // sfm_ctx_opts.flags (the SFM_CTX_BA_* engine shape)
    // engine shape decoded from the flags: lanes per point in the step pass,
    // waves per reduce target (0: the plan chooses)
    int step_lanes() const {
        const int v = (flags >> 12) & 7;
        return v ? 1 << (v - 1) : 0;
    }
    int reduce_waves() const {
        const int v = (flags >> 15) & 7;
        return v ? 1 << (v - 1) : 0;
    }
    hipEvent_t ev[2] = {nullptr, nullptr};       // timing events, created on first use
    double last_kernel_ms = -1.0;                // sfm_fmatrix_ac's kernel (sfm_ctx_last_kernel_ms)
    // sfm_ba_solve's plan cache: plans reused as they were / grown from the
    // cached one / built from scratch (sfm_ba_cache_stats)
    int64_t plans_reused = 0, plans_grown = 0, plans_fresh = 0;
};

namespace sfm {
// releases the context's cached BA plan (ba_solver.cpp; sfm_ctx_destroy)
void ba_cache_release(sfm_ctx* ctx);
// the context's two timing events (created once, destroyed with the context)
inline hipEvent_t* ctx_events(sfm_ctx* ctx) {
    if (!ctx->ev[0]) {
        SFM_HIP(hipEventCreate(&ctx->ev[0]));
        SFM_HIP(hipEventCreate(&ctx->ev[1]));
    }
    return ctx->ev;
}
}  // namespace sfm
