// hip_util.h -- small HIP helpers shared by the ipo-hip sources.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace ipo {

struct HipError : std::runtime_error {
    explicit HipError(const std::string& s) : std::runtime_error(s) {}
};

#define IPO_HIP_CHECK(expr)                                                           \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            throw ::ipo::HipError(std::string(#expr) + " failed: " + hipGetErrorString(e_) + \
                                  " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    } while (0)

// Owning device allocation.
template <typename T>
class DevBuf {
  public:
    DevBuf() = default;
    explicit DevBuf(size_t n) { alloc(n); }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
        return *this;
    }
    void alloc(size_t n) {
        release();
        n_ = n;
        if (n) IPO_HIP_CHECK(hipMalloc(&p_, n * sizeof(T)));
    }
    void release() {
        if (p_) (void)hipFree(p_);
        p_ = nullptr;
        n_ = 0;
    }
    void upload(const T* h, size_t n, hipStream_t s) {
        if (n > n_) alloc(n);
        if (n) IPO_HIP_CHECK(hipMemcpyAsync(p_, h, n * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void upload(const std::vector<T>& v, hipStream_t s) { upload(v.data(), v.size(), s); }
    void download(T* h, size_t n, hipStream_t s) const {
        if (n) IPO_HIP_CHECK(hipMemcpyAsync(h, p_, n * sizeof(T), hipMemcpyDeviceToHost, s));
    }
    T* get() const { return p_; }
    size_t size() const { return n_; }
    size_t bytes() const { return n_ * sizeof(T); }

  private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

inline int ceil_div(long a, long b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace ipo
