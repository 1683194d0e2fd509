// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against known
// byte counts, for the access widths the PA kernels use (profiling infrastructure, not product).
// Each kernel touches a buffer of 1 GiB (4x the 256 MiB Infinity Cache), every byte once, so
// the true DRAM traffic is the byte count the name states; one dispatch per kernel, in order:
//   rd16  16 B/lane coalesced streaming read       (global_load_dwordx4)
//   rd8    8 B/lane coalesced streaming read       (global_load_dwordx2: x gathers, partials)
//   rd4    4 B/lane coalesced streaming read       (global_load_dword: maps)
//   rdl8   8 B per 128-B line, one lane per line   (a sparse gather: 1/16 of the line used)
//   wr8    8 B/lane coalesced streaming store      (y / partial-slot stores)
//   wr16  16 B/lane coalesced streaming store
// profiles/calib/run_calib.sh runs it under separate FETCH_SIZE and WRITE_SIZE passes and
// profiles/calib/calib_reduce.py divides the counters by the known bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ void rd16(const v2d *__restrict__ a, long n, double *out)
{
   v2d s = {0.0, 0.0};
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { s += a[i]; }
   if (s.x + s.y == 1.2345e300) { out[0] = s.x; }  // never: keeps the loads
}
__global__ void rd8(const double *__restrict__ a, long n, double *out)
{
   double s = 0.0;
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { s += a[i]; }
   if (s == 1.2345e300) { out[0] = s; }
}
__global__ void rd4(const int *__restrict__ a, long n, double *out)
{
   int s = 0;
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { s ^= a[i]; }
   if (s == 0x7eadbeef) { out[0] = s; }
}
__global__ void rdl8(const double *__restrict__ a, long nlines, double *out)
{
   double s = 0.0;
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nlines; i += (long)gridDim.x * blockDim.x) { s += a[i * 16]; }
   if (s == 1.2345e300) { out[0] = s; }
}
__global__ void wr8(double *__restrict__ a, long n)
{
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { a[i] = (double)i; }
}
__global__ void wr16(v2d *__restrict__ a, long n)
{
   for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { a[i] = v2d{(double)i, 1.0}; }
}

int main()
{
   const long bytes = 1L << 30;
   char *buf = nullptr;
   double *out = nullptr;
   CK(hipMalloc(&buf, bytes));
   CK(hipMalloc(&out, 64));
   CK(hipMemset(buf, 0, bytes));
   // evict the buffer's tail from the Infinity Cache: stream a second 512 MiB buffer
   char *flush = nullptr;
   CK(hipMalloc(&flush, bytes / 2));
   const dim3 g(256 * 8 * 4), b(256);
   auto evict = [&] { hipLaunchKernelGGL(wr8, g, b, 0, 0, (double *)flush, bytes / 2 / 8); };
   evict();
   hipLaunchKernelGGL(rd16, g, b, 0, 0, (const v2d *)buf, bytes / 16, out);
   evict();
   hipLaunchKernelGGL(rd8, g, b, 0, 0, (const double *)buf, bytes / 8, out);
   evict();
   hipLaunchKernelGGL(rd4, g, b, 0, 0, (const int *)buf, bytes / 4, out);
   evict();
   hipLaunchKernelGGL(rdl8, g, b, 0, 0, (const double *)buf, bytes / 128, out);
   evict();
   hipLaunchKernelGGL(wr8, g, b, 0, 0, (double *)buf, bytes / 8);
   evict();
   hipLaunchKernelGGL(wr16, g, b, 0, 0, (v2d *)buf, bytes / 16);
   CK(hipDeviceSynchronize());
   std::printf("{\"bytes\": %ld, \"rd16\": %ld, \"rd8\": %ld, \"rd4\": %ld, \"rdl8_lines\": %ld, \"rdl8_bytes_used\": %ld, \"wr8\": %ld, \"wr16\": %ld}\n",
               bytes, bytes, bytes, bytes, bytes / 128, bytes / 16, bytes, bytes);
   CK(hipFree(flush));
   CK(hipFree(buf));
   CK(hipFree(out));
   return 0;
}
