// Probe (round 5): the deterministic dot of the device PCG at a rank's and a whole GPU's size.
//   two    : k_dot_partial over 1024 workgroups + a one-workgroup k_dot_final (rounds 1-4)
//   flat   : one pass, each workgroup parks its sum (agent-scope write-through store, acknowledged)
//            and arrives on ONE counter; the last sums the parks (the library's k_dot at 6e1c... )
//   xcd    : one pass, arrivals first on one of 8 counters (blockIdx % 8: the workgroup's XCD under
//            round-robin dispatch), the last of each group then on a top counter
//   blocksN: 'flat' with N workgroups (fewer arrivals, more elements per thread)
// Each variant: 200 back-to-back launches timed with HIP events; result checked bitwise against 'two'
// (same reduction order) or against a long-double host sum (other grids).
// Build: hipcc --offload-arch=gfx950 -O3 -o profiles/calib/dot_probe profiles/calib/dot_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
   do {                                                                                        \
      hipError_t e_ = (x);                                                                     \
      if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } \
   } while (0)

__device__ __forceinline__ double wg_sum(double s, double *red)
{
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   const double v = (red[0] + red[1]) + (red[2] + red[3]);
   __syncthreads();
   return v;
}

__device__ __forceinline__ double grid_stride(int n, const double *a, const double *b)
{
   double s = 0.0;
   for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
   {
      s += a[i] * b[i];
   }
   return s;
}

__global__ void __launch_bounds__(256) k_partial(int n, const double *a, const double *b, double *parts)
{
   __shared__ double red[4];
   const double v = wg_sum(grid_stride(n, a, b), red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

// the grid-stride loop unrolled by 4: the loads of four strides issued before the first
// accumulation, the accumulation in the same order (bitwise the same sum as k_partial)
__global__ void __launch_bounds__(256) k_partial_u4(int n, const double *__restrict__ a, const double *__restrict__ b,
                                                    double *parts)
{
   __shared__ double red[4];
   const long G = (long)gridDim.x * blockDim.x;
   long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   double s = 0.0;
   for (; i + 3 * G < n; i += 4 * G)
   {
      const double a0 = a[i], a1 = a[i + G], a2 = a[i + 2 * G], a3 = a[i + 3 * G];
      const double b0 = b[i], b1 = b[i + G], b2 = b[i + 2 * G], b3 = b[i + 3 * G];
      s += a0 * b0;
      s += a1 * b1;
      s += a2 * b2;
      s += a3 * b3;
   }
   for (; i < n; i += G) { s += a[i] * b[i]; }
   const double v = wg_sum(s, red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

// the PCG update's shape (x += al d, r -= al z, z = dinv r, sum r z): plain and unrolled by 4
__global__ void __launch_bounds__(256) k_step(int n, double al, const double *__restrict__ d, double *__restrict__ z,
                                              double *__restrict__ x, double *__restrict__ r,
                                              const double *__restrict__ dinv, double *parts)
{
   __shared__ double red[4];
   double s = 0.0;
   for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
   {
      x[i] = x[i] + al * d[i];
      const double rn = r[i] + (-al) * z[i];
      r[i] = rn;
      const double zn = dinv[i] * rn;
      z[i] = zn;
      s += rn * zn;
   }
   const double v = wg_sum(s, red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

__global__ void __launch_bounds__(256) k_step_u4(int n, double al, const double *__restrict__ d, double *__restrict__ z,
                                                 double *__restrict__ x, double *__restrict__ r,
                                                 const double *__restrict__ dinv, double *parts)
{
   __shared__ double red[4];
   const long G = (long)gridDim.x * blockDim.x;
   long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   double s = 0.0;
   for (; i + 3 * G < n; i += 4 * G)
   {
      double xv[4], dv[4], rv[4], zv[4], iv[4];
#pragma unroll
      for (int k = 0; k < 4; k++)
      {
         xv[k] = x[i + k * G]; dv[k] = d[i + k * G]; rv[k] = r[i + k * G]; zv[k] = z[i + k * G]; iv[k] = dinv[i + k * G];
      }
#pragma unroll
      for (int k = 0; k < 4; k++)
      {
         x[i + k * G] = xv[k] + al * dv[k];
         const double rn = rv[k] + (-al) * zv[k];
         r[i + k * G] = rn;
         const double zn = iv[k] * rn;
         z[i + k * G] = zn;
         s += rn * zn;
      }
   }
   for (; i < n; i += G)
   {
      x[i] = x[i] + al * d[i];
      const double rn = r[i] + (-al) * z[i];
      r[i] = rn;
      const double zn = dinv[i] * rn;
      z[i] = zn;
      s += rn * zn;
   }
   const double v = wg_sum(s, red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

__global__ void __launch_bounds__(256) k_final(int np, const double *parts, double *out)
{
   __shared__ double red[4];
   double t = 0.0;
   for (int i = threadIdx.x; i < np; i += blockDim.x) { t += parts[i]; }
   const double v = wg_sum(t, red);
   if (threadIdx.x == 0) { *out = v; }
}

__device__ __forceinline__ void finish(double v, double *parts, double *out, double *red)
{
   double t = 0.0;
   for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
   {
      t += __hip_atomic_load(parts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   }
   const double r = wg_sum(t, red);
   if (threadIdx.x == 0) { *out = r; }
   (void)v;
}

__global__ void __launch_bounds__(256) k_flat(int n, const double *a, const double *b, double *parts, unsigned *cnt,
                                              double *out)
{
   __shared__ double red[4];
   __shared__ int last;
   const double v = wg_sum(grid_stride(n, a, b), red);
   if (threadIdx.x == 0)
   {
      __hip_atomic_store(parts + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
   }
   __syncthreads();
   if (!last) { return; }
   finish(v, parts, out, red);
   if (threadIdx.x == 0) { __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
}

__global__ void __launch_bounds__(256) k_xcd(int n, const double *a, const double *b, double *parts, unsigned *cnt,
                                             double *out)
{
   __shared__ double red[4];
   __shared__ int last;
   const double v = wg_sum(grid_stride(n, a, b), red);
   if (threadIdx.x == 0)
   {
      __hip_atomic_store(parts + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned g = blockIdx.x & 7, members = (gridDim.x - g + 7) / 8;
      int l = __hip_atomic_fetch_add(cnt + 16 * (1 + g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1;
      if (l)
      {
         __hip_atomic_store(cnt + 16 * (1 + g), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         l = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 7;
      }
      last = l;
   }
   __syncthreads();
   if (!last) { return; }
   finish(v, parts, out, red);
   if (threadIdx.x == 0) { __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
}

typedef double v2d __attribute__((ext_vector_type(2)));

// the update's shape with two elements per thread (16-byte accesses), r.z summed in element order
__global__ void __launch_bounds__(256) k_step_v2(int n, double al, const double *__restrict__ d, double *__restrict__ z,
                                                 double *__restrict__ x, double *__restrict__ r,
                                                 const double *__restrict__ dinv, double *parts)
{
   __shared__ double red[4];
   double s = 0.0;
   const int n2 = n / 2;
   for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < n2; p += (long)gridDim.x * blockDim.x)
   {
      const v2d xv = reinterpret_cast<const v2d *>(x)[p], dv = reinterpret_cast<const v2d *>(d)[p];
      const v2d rv = reinterpret_cast<const v2d *>(r)[p], zv = reinterpret_cast<const v2d *>(z)[p];
      const v2d iv = reinterpret_cast<const v2d *>(dinv)[p];
      reinterpret_cast<v2d *>(x)[p] = xv + al * dv;
      const v2d rn = rv + (-al) * zv;
      reinterpret_cast<v2d *>(r)[p] = rn;
      const v2d zn = iv * rn;
      reinterpret_cast<v2d *>(z)[p] = zn;
      s += rn.x * zn.x;
      s += rn.y * zn.y;
   }
   const double v = wg_sum(s, red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

__global__ void k_upd(int n, double be, const double *__restrict__ z, double *__restrict__ d)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { d[i] = z[i] + be * d[i]; }
}

__global__ void k_upd_v2(int n2, double be, const double *__restrict__ z, double *__restrict__ d)
{
   const int p = blockIdx.x * blockDim.x + threadIdx.x;
   if (p < n2)
   {
      const v2d zv = reinterpret_cast<const v2d *>(z)[p], dv = reinterpret_cast<const v2d *>(d)[p];
      reinterpret_cast<v2d *>(d)[p] = zv + be * dv;
   }
}

__global__ void __launch_bounds__(256) k_partial_v2(int n, const double *__restrict__ a, const double *__restrict__ b,
                                                    double *parts)
{
   __shared__ double red[4];
   double s = 0.0;
   for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < n / 2; p += (long)gridDim.x * blockDim.x)
   {
      const v2d av = reinterpret_cast<const v2d *>(a)[p], bv = reinterpret_cast<const v2d *>(b)[p];
      s += av.x * bv.x;
      s += av.y * bv.y;
   }
   const double v = wg_sum(s, red);
   if (threadIdx.x == 0) { parts[blockIdx.x] = v; }
}

int main()
{
   const int sizes[2] = {1277289, 10218313};  // an N = 8 rank's true dofs (C4), the whole C4 space
   double *a, *b, *parts, *out;
   unsigned *cnt;
   CK(hipMalloc(&a, sizeof(double) * sizes[1]));
   CK(hipMalloc(&b, sizeof(double) * sizes[1]));
   CK(hipMalloc(&parts, sizeof(double) * 4096));
   CK(hipMalloc(&out, sizeof(double) * 8));
   CK(hipMalloc(&cnt, sizeof(unsigned) * 16 * 9));
   CK(hipMemset(cnt, 0, sizeof(unsigned) * 16 * 9));
   std::vector<double> ha(sizes[1]), hb(sizes[1]);
   srand(7);
   for (int i = 0; i < sizes[1]; i++)
   {
      ha[i] = rand() / (double)RAND_MAX - 0.5;
      hb[i] = rand() / (double)RAND_MAX - 0.5;
   }
   CK(hipMemcpy(a, ha.data(), sizeof(double) * sizes[1], hipMemcpyHostToDevice));
   CK(hipMemcpy(b, hb.data(), sizeof(double) * sizes[1], hipMemcpyHostToDevice));
   hipEvent_t e0, e1;
   CK(hipEventCreate(&e0));
   CK(hipEventCreate(&e1));
   const int reps = 200;
   for (int n : sizes)
   {
      long double ref = 0;
      for (int i = 0; i < n; i++) { ref += (long double)ha[i] * hb[i]; }
      double two_val = 0;
      auto run = [&](const char *name, auto launch) {
         for (int w = 0; w < 20; w++) { launch(); }
         CK(hipDeviceSynchronize());
         CK(hipEventRecord(e0));
         for (int r = 0; r < reps; r++) { launch(); }
         CK(hipEventRecord(e1));
         CK(hipEventSynchronize(e1));
         float ms = 0;
         CK(hipEventElapsedTime(&ms, e0, e1));
         double v = 0;
         CK(hipMemcpy(&v, out, sizeof(double), hipMemcpyDeviceToHost));
         if (std::string(name) == "two") { two_val = v; }
         std::printf("n=%9d %-10s %8.2f us/launch  %6.2f TB/s  value %.17g  bitwise_vs_two %d  relerr_vs_longdouble %.2e\n",
                     n, name, ms * 1e3 / reps, 16.0 * n / (ms * 1e-3 / reps) / 1e12, v, v == two_val,
                     (double)std::fabs((long double)v - ref) / (double)std::fabs(ref));
      };
      run("two", [&] {
         hipLaunchKernelGGL(k_partial, dim3(1024), dim3(256), 0, 0, n, a, b, parts);
         hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, 1024, parts, out);
      });
      run("two_v2", [&] {
         hipLaunchKernelGGL(k_partial_v2, dim3(1024), dim3(256), 0, 0, n, a, b, parts);
         hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, 1024, parts, out);
      });
      run("two_u4", [&] {
         hipLaunchKernelGGL(k_partial_u4, dim3(1024), dim3(256), 0, 0, n, a, b, parts);
         hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, 1024, parts, out);
      });
      for (int nb : {1024, 2048, 4096})
      {
         char nm[32];
         std::snprintf(nm, sizeof nm, "two_u4_%d", nb);
         run(nm, [&] {
            hipLaunchKernelGGL(k_partial_u4, dim3(nb), dim3(256), 0, 0, n, a, b, parts);
            hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, nb, parts, out);
         });
      }
      // the update's shape on five work vectors (x, r, z, d, dinv): 8 streams per element
      {
         double *x5;
         CK(hipMalloc(&x5, sizeof(double) * 3 * (size_t)n));
         CK(hipMemset(x5, 0, sizeof(double) * 3 * (size_t)n));
         auto step = [&](const char *name, auto kern, int nb) {
            for (int w = 0; w < 10; w++) { hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, n, 1e-3, a, x5, x5 + n, x5 + 2 * (size_t)n, b, parts); }
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++)
            {
               hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, n, 1e-3, a, x5, x5 + n, x5 + 2 * (size_t)n, b, parts);
               hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, nb, parts, out);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("n=%9d %-12s %8.2f us/launch  %6.2f TB/s (8 streams)\n", n, name, ms * 1e3 / reps,
                        64.0 * n / (ms * 1e-3 / reps) / 1e12);
         };
         step("step", k_step, 1024);
         step("step_v2", k_step_v2, 1024);
         step("step_v2_512", k_step_v2, 512);
         {
            auto upd = [&](const char *name, auto launch) {
               for (int w = 0; w < 10; w++) { launch(); }
               CK(hipDeviceSynchronize());
               CK(hipEventRecord(e0));
               for (int r = 0; r < reps; r++) { launch(); }
               CK(hipEventRecord(e1));
               CK(hipEventSynchronize(e1));
               float ms = 0;
               CK(hipEventElapsedTime(&ms, e0, e1));
               std::printf("n=%9d %-12s %8.2f us/launch  %6.2f TB/s (3 streams)\n", n, name, ms * 1e3 / reps,
                           24.0 * n / (ms * 1e-3 / reps) / 1e12);
            };
            upd("upd", [&] { hipLaunchKernelGGL(k_upd, dim3((n + 255) / 256), dim3(256), 0, 0, n, 0.5, a, x5); });
            upd("upd_v2", [&] { hipLaunchKernelGGL(k_upd_v2, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, n / 2, 0.5, a, x5); });
         }
         step("step_u4", k_step_u4, 1024);
         step("step_u4_2k", k_step_u4, 2048);
         step("step_4k", k_step, 4096);
         CK(hipFree(x5));
      }
      run("flat", [&] { hipLaunchKernelGGL(k_flat, dim3(1024), dim3(256), 0, 0, n, a, b, parts, cnt, out); });
      run("xcd", [&] { hipLaunchKernelGGL(k_xcd, dim3(1024), dim3(256), 0, 0, n, a, b, parts, cnt, out); });
      for (int nb : {256, 512, 2048})
      {
         char nm[32];
         std::snprintf(nm, sizeof nm, "flat%d", nb);
         run(nm, [&] { hipLaunchKernelGGL(k_flat, dim3(nb), dim3(256), 0, 0, n, a, b, parts, cnt, out); });
      }
      for (int nb : {256, 512})
      {
         char nm[32];
         std::snprintf(nm, sizeof nm, "two%d", nb);
         run(nm, [&] {
            hipLaunchKernelGGL(k_partial, dim3(nb), dim3(256), 0, 0, n, a, b, parts);
            hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, 0, nb, parts, out);
         });
      }
   }
   std::printf("done\n");
   return 0;
}
