// common.hpp -- error handling, HIP checks and device buffers for the ecm2 PA library.
//
// Error convention mirrors the reference's MFEM_VERIFY -> mfem_error path
// (general/error.hpp:104-125, error.cpp:154-184): a failed check is fatal for
// the operation.  Inside the library it throws ecm2::Error; the C ABI
// (capi.cpp) catches it, records the message for ecm2_last_error() and returns
// a nonzero status.  No CPU fallback exists anywhere: a missing GPU or HIP
// failure is reported, never papered over.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace ecm2
{

struct Error : std::runtime_error
{
   int code;
   Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

enum Status : int
{
   OK = 0,
   ERR_ARG = 1,       // invalid argument / shape
   ERR_HIP = 2,       // HIP runtime failure (incl. no device)
   ERR_STATE = 3,     // call order violated (e.g. Mult before Assemble)
   ERR_IO = 4,        // mesh file problems
   ERR_UNSUPPORTED = 5,
   ERR_COMM = 6,      // RCCL failure
   ERR_INTERNAL = 7,
   ERR_NUMERIC = 8    // non-finite value where the reference's MFEM_VERIFY(IsFinite) aborts
};

#define ECM2_VERIFY(cond, code, msg)                                          \
   do {                                                                       \
      if (!(cond)) {                                                          \
         std::ostringstream ecm2_os_;                                         \
         ecm2_os_ << msg << " [" << __FILE__ << ":" << __LINE__ << "]";       \
         throw ::ecm2::Error((code), ecm2_os_.str());                         \
      }                                                                       \
   } while (0)

#define ECM2_HIP(call)                                                        \
   do {                                                                       \
      hipError_t ecm2_e_ = (call);                                            \
      if (ecm2_e_ != hipSuccess) {                                            \
         std::ostringstream ecm2_os_;                                         \
         ecm2_os_ << "HIP error '" << hipGetErrorString(ecm2_e_) << "' in "  \
                  << #call << " [" << __FILE__ << ":" << __LINE__ << "]";     \
         throw ::ecm2::Error(::ecm2::ERR_HIP, ecm2_os_.str());                \
      }                                                                       \
   } while (0)

// Owning device allocation (hipMalloc'd, freed on destruction).
template <typename T>
class DeviceArray
{
public:
   DeviceArray() = default;
   explicit DeviceArray(size_t n) { resize(n); }
   DeviceArray(const DeviceArray &) = delete;
   DeviceArray &operator=(const DeviceArray &) = delete;
   DeviceArray(DeviceArray &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
   DeviceArray &operator=(DeviceArray &&o) noexcept
   {
      if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
      return *this;
   }
   ~DeviceArray() { release(); }

   void resize(size_t n)
   {
      if (n == n_) { return; }
      release();
      if (n) { ECM2_HIP(hipMalloc(&p_, n * sizeof(T))); }
      n_ = n;
   }
   void upload(const T *h, size_t n, hipStream_t s = nullptr)
   {
      resize(n);
      if (n) { ECM2_HIP(hipMemcpyAsync(p_, h, n * sizeof(T), hipMemcpyHostToDevice, s)); }
   }
   void upload(const std::vector<T> &h, hipStream_t s = nullptr) { upload(h.data(), h.size(), s); }
   void download(T *h, hipStream_t s = nullptr) const
   {
      if (n_) { ECM2_HIP(hipMemcpyAsync(h, p_, n_ * sizeof(T), hipMemcpyDeviceToHost, s)); }
      ECM2_HIP(hipStreamSynchronize(s));
   }
   T *data() { return p_; }
   const T *data() const { return p_; }
   size_t size() const { return n_; }
   size_t bytes() const { return n_ * sizeof(T); }

private:
   void release()
   {
      if (p_) { (void)hipFree(p_); }
      p_ = nullptr;
      n_ = 0;
   }
   T *p_ = nullptr;
   size_t n_ = 0;
};

// Throws ERR_HIP if no usable GPU is present: the product path has no CPU fallback.
void require_device();

} // namespace ecm2
