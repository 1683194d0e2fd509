// k_misc.hip -- reference-shaped pieces and vector kernels (gfx950): the workgroup-per-element
// apply (E-vector AddMultPA, unfused Mult), ElementRestriction, the generic diagonal, the
// deterministic summation pass of the fused kernels' scatter, halo pack/unpack, and the
// device PCG / ODE vector kernels.
#include "dev_common.hpp"

#include <algorithm>

namespace ecm2
{
namespace
{
using namespace dev;
using kern::PcgCtl;
using kern::PCG_RUNNING;
using kern::PCG_CONVERGED;
using kern::PCG_MAX_ITER;
using kern::PCG_NEG_BR;
using kern::PCG_DEN_ZERO;
using kern::PCG_NONFINITE;

// Workgroup per element (lane per quadrature point), any layout, L- or E-vectors in and
// out (in_e / out_e): six 1D stages through LDS, the reference's smem kernels' structure
// (bilininteg_mass_kernels.hpp:809-1033, bilininteg_diffusion_kernels.hpp:989-1214).
template <int D, int Q, bool MASS, bool DIFF>
__global__ void k_apply_wpe(const int *__restrict__ pos, int kind, int ne, int e_begin, int n_owned,
                            const int *__restrict__ gmap,
                            const double *__restrict__ qdd, const double *__restrict__ qdm,
                            const double *__restrict__ x, const double *__restrict__ xg,
                            double *__restrict__ y, double *__restrict__ yg, const Basis1D b, bool in_e,
                            bool out_e)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q;
   __shared__ double sB[Q * D], sG[Q * D];
   __shared__ double sX[ND];
   __shared__ double s1a[D * D * Q], s1b[D * D * Q];
   __shared__ double s2a[D * Q * Q], s2b[D * Q * Q], s2c[D * Q * Q];
   __shared__ double s3m[NQ], s3x[NQ], s3y[NQ], s3z[NQ];
   __shared__ double s4a[Q * Q * D], s4b[Q * Q * D], s4c[Q * Q * D];
   __shared__ double s5a[Q * D * D], s5b[Q * D * D];
   const int e = e_begin + blockIdx.x;
   const int t = threadIdx.x;
   if (t < Q * D)
   {
      const int q = t % Q, d = t / Q;
      sB[q + Q * d] = b.B[q + MQ * d];
      sG[q + Q * d] = b.G[q + MQ * d];
   }
   if (t < ND)
   {
      if (in_e) { sX[t] = x[(size_t)e * ND + t]; }
      else
      {
         const int g = gmap[(size_t)e * ND + t];
         const int d = dof_of(g);
         const double v = d < n_owned ? x[d] : xg[d - n_owned];
         sX[t] = g >= 0 ? v : -v;
      }
   }
   __syncthreads();
   // stage 1: x-contraction  (qx, dy, dz)
   if (t < D * D * Q)
   {
      const int qx = t % Q, dy = (t / Q) % D, dz = t / (Q * D);
      double u = 0.0, v = 0.0;
      for (int dx = 0; dx < D; dx++)
      {
         const double c = sX[(dz * D + dy) * D + dx];
         u += c * sB[qx + Q * dx];
         v += c * sG[qx + Q * dx];
      }
      s1a[t] = u;  // B_x
      s1b[t] = v;  // G_x
   }
   __syncthreads();
   // stage 2: y-contraction  (qx, qy, dz)
   if (t < D * Q * Q)
   {
      const int qx = t % Q, qy = (t / Q) % Q, dz = t / (Q * Q);
      double u = 0.0, v = 0.0, w = 0.0;
      for (int dy = 0; dy < D; dy++)
      {
         const int i = (dz * D + dy) * Q + qx;
         u += s1b[i] * sB[qy + Q * dy];   // G_x B_y
         v += s1a[i] * sG[qy + Q * dy];   // B_x G_y
         w += s1a[i] * sB[qy + Q * dy];   // B_x B_y
      }
      s2a[t] = u; s2b[t] = v; s2c[t] = w;
   }
   __syncthreads();
   // stage 3: z-contraction + pointwise qdata (qx, qy, qz)
   if (t < NQ)
   {
      const int qx = t % Q, qy = (t / Q) % Q, qz = t / (Q * Q);
      double gx = 0.0, gy = 0.0, gz = 0.0, u = 0.0;
      for (int dz = 0; dz < D; dz++)
      {
         const int i = (dz * Q + qy) * Q + qx;
         gx += s2a[i] * sB[qz + Q * dz];
         gy += s2b[i] * sB[qz + Q * dz];
         gz += s2c[i] * sG[qz + Q * dz];
         u += s2c[i] * sB[qz + Q * dz];
      }
      double m = 0.0, fx = 0.0, fy = 0.0, fz = 0.0;
      if (MASS) { m = qd_mass_at(qdm, pos, kind, NQ, e, t) * u; }
      if (DIFF)
      {
         // (11,12,13,22,23,33), or NATIVE9's general D_ij at 3 i + j (SmemPADiffusionApply3D,
         // bilininteg_diffusion_kernels.hpp:1122-1136: "symmetric ? ... : d(q, 3..8)")
         const bool g9 = kind == QLAYOUT_NATIVE9;
         const double O11 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 0, t);
         const double O12 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 1, t);
         const double O13 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 2, t);
         const double O21 = g9 ? qd_diff_at(qdd, qdm, pos, kind, NQ, e, 3, t) : O12;
         const double O22 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, g9 ? 4 : 3, t);
         const double O23 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, g9 ? 5 : 4, t);
         const double O31 = g9 ? qd_diff_at(qdd, qdm, pos, kind, NQ, e, 6, t) : O13;
         const double O32 = g9 ? qd_diff_at(qdd, qdm, pos, kind, NQ, e, 7, t) : O23;
         const double O33 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, g9 ? 8 : 5, t);
         fx = (O11 * gx) + (O12 * gy) + (O13 * gz);
         fy = (O21 * gx) + (O22 * gy) + (O23 * gz);
         fz = (O31 * gx) + (O32 * gy) + (O33 * gz);
      }
      s3m[t] = m; s3x[t] = fx; s3y[t] = fy; s3z[t] = fz;
   }
   __syncthreads();
   // stage 4: x-transpose (dx, qy, qz)
   if (t < Q * Q * D)
   {
      const int dx = t % D, qy = (t / D) % Q, qz = t / (D * Q);
      double u = 0.0, v = 0.0, w = 0.0;
      for (int qx = 0; qx < Q; qx++)
      {
         const int i = (qz * Q + qy) * Q + qx;
         u += s3x[i] * sG[qx + Q * dx] + s3m[i] * sB[qx + Q * dx];
         v += s3y[i] * sB[qx + Q * dx];
         w += s3z[i] * sB[qx + Q * dx];
      }
      s4a[t] = u; s4b[t] = v; s4c[t] = w;
   }
   __syncthreads();
   // stage 5: y-transpose (dx, dy, qz)
   if (t < Q * D * D)
   {
      const int dx = t % D, dy = (t / D) % D, qz = t / (D * D);
      double u = 0.0, w = 0.0;
      for (int qy = 0; qy < Q; qy++)
      {
         const int i = (qz * Q + qy) * D + dx;
         u += s4a[i] * sB[qy + Q * dy] + s4b[i] * sG[qy + Q * dy];
         w += s4c[i] * sB[qy + Q * dy];
      }
      s5a[t] = u; s5b[t] = w;
   }
   __syncthreads();
   // stage 6: z-transpose (dx, dy, dz) + output
   if (t < ND)
   {
      const int dx = t % D, dy = (t / D) % D, dz = t / (D * D);
      double u = 0.0;
      for (int qz = 0; qz < Q; qz++)
      {
         const int i = (qz * D + dy) * D + dx;
         u += s5a[i] * sB[qz + Q * dz] + s5b[i] * sG[qz + Q * dz];
      }
      if (out_e) { y[(size_t)e * ND + t] += u; }
      else
      {
         const int g = gmap[(size_t)e * ND + t];
         const int d = dof_of(g);
         double *dst = d < n_owned ? y + d : yg + (d - n_owned);
         unsafeAtomicAdd(dst, g >= 0 ? u : -u);
      }
   }
}

__global__ void k_restriction_mult(long n, const int *__restrict__ gmap,
                                   const double *__restrict__ x, double *__restrict__ xe)
{
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= n) { return; }
   const int g = gmap[i];
   const double v = x[dof_of(g)];
   xe[i] = g >= 0 ? v : -v;
}

__global__ void k_restriction_mult_transpose(int ndofs, const int *__restrict__ offsets,
                                             const int *__restrict__ indices,
                                             const double *__restrict__ xe,
                                             double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= ndofs) { return; }
   double v = 0.0;
   for (int j = offsets[i]; j < offsets[i + 1]; j++)
   {
      const int idx = indices[j];
      v += idx >= 0 ? xe[idx] : -xe[-1 - idx];
   }
   y[i] = v;
}

// Diagonal, one thread per (element, dof): the direct (not sum-factorised) sum over the
// quadrature points, for (D1D, Q1D) pairs the sum-factorised kernel does not instantiate.
__global__ void k_diagonal(const int *__restrict__ pos, int D, int Q, int kind, int ne, const int *__restrict__ gmap,
                           const double *__restrict__ qdd, const double *__restrict__ qdm,
                           double *__restrict__ diag, bool out_e, const Basis1D b)
{
   const int ND = D * D * D, NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * ND) { return; }
   const int e = (int)(t / ND), a = (int)(t % ND);
   const int dx = a % D, dy = (a / D) % D, dz = a / (D * D);
   double s = 0.0;
   for (int qz = 0; qz < Q; qz++)
      for (int qy = 0; qy < Q; qy++)
         for (int qx = 0; qx < Q; qx++)
         {
            const int q = (qz * Q + qy) * Q + qx;
            const double bx = b.B[qx + MQ * dx], by = b.B[qy + MQ * dy], bz = b.B[qz + MQ * dz];
            const double gx = b.G[qx + MQ * dx], gy = b.G[qy + MQ * dy], gz = b.G[qz + MQ * dz];
            if (qdm) { s += bx * bx * by * by * bz * bz * qd_mass_at(qdm, pos, kind, NQ, e, q); }
            if (qdd)
            {
               const double p0 = gx * by * bz, p1 = bx * gy * bz, p2 = bx * by * gz;
               s += p0 * p0 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 0, q) +
                    p1 * p1 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 1, q) +
                    p2 * p2 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 2, q) +
                    (p0 * p1 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 3, q) +
                     p0 * p2 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 4, q) +
                     p1 * p2 * qd_diag_term(qdd, qdm, pos, kind, NQ, e, 5, q));
            }
         }
   if (out_e) { diag[t] += s; }
   else { unsafeAtomicAdd(diag + dof_of(gmap[t]), s); }
}

__global__ void k_set_values(int n, const int *__restrict__ idx, double val, double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[idx[i]] = val; }
}

__global__ void k_copy_values(int n, const int *__restrict__ idx, const double *__restrict__ x,
                              double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[idx[i]] = x[idx[i]]; }
}


// CGSolver's stopping tests (solvers.cpp:950-1000) as the device-driven loop runs them.
// kind 0: the test of iteration `it` on betanom = (B r, r): not finite -> MFEM_VERIFY's abort
// (PCG_NONFINITE, the host raises ECM2_ERR_NUMERIC); < 0 -> not converged (the preconditioner is not
// positive definite, :955-964); <= r0 -> converged (:972-977); it + 1 > max_iter -> stopped (:979-982).
// kind 1: the test of den = (A d, d) in iteration it's tail, after ++i (`it` is then the next
// iteration's number, :993-1004): not finite -> abort; == 0 -> stopped, not converged, final_iter = it.
struct PcgCheck
{
   double r0;
   int it, max_iter;
   PcgCtl *ctl, *host;
   const double *betanom;
   int kind;
};

__device__ void pcg_check_one(double v, const PcgCheck &c)
{
   if (c.ctl->done) { return; }
   int done;
   double fin = v;
   if (c.kind == 0)
   {
      done = !isfinite(v) ? PCG_NONFINITE
             : v < 0.0    ? PCG_NEG_BR
             : v <= c.r0  ? PCG_CONVERGED
             : (c.it + 1 > c.max_iter ? PCG_MAX_ITER : PCG_RUNNING);
   }
   else
   {
      done = !isfinite(v) ? PCG_NONFINITE : (v == 0.0 ? PCG_DEN_ZERO : PCG_RUNNING);
      fin = *c.betanom;  // (final_norm = sqrt(betanom) of the iteration, :1047)
   }
   if (done)
   {
      c.ctl->done = done;
      c.ctl->iters = c.it;
      c.ctl->final = fin;
      c.host->final = fin;
      c.host->iters = c.it;
      __threadfence_system();  // (the mirror's fields before its flag)
      c.host->done = done;
   }
   if (c.kind == 0)
   {
      __threadfence_system();  // (the flag before the progress mark the host polls)
      c.host->checked = c.it;
   }
}

// Deterministic dot, pass 1: each workgroup writes its sum (a fixed order per workgroup).  (A
// one-pass form -- the last workgroup to arrive on a counter sums the parks -- was measured slower:
// the 1,024 arrivals on one counter serialise, 16.6 vs 6.5 us per dot at a rank's 1.28M dofs,
// profiles/r5/dot_probe.txt.)
__device__ __forceinline__ void dot_park(double s, double *__restrict__ partials)
{
   __shared__ double red[4];
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   if (threadIdx.x == 0) { partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]); }
}

// (ctl: read only when no check writes it in the same kernel -- no __restrict__ on it)
// A flat grid of contiguous chunks: workgroup b sums pairs [b kStepChunk, (b + 1) kStepChunk) -- grid-stride
// loops stream 15-35% slower on this chip (profiles/r6/copy_probe.json: a 16-byte copy 6.67 TB/s flat against
// 4.4-5.4 TB/s grid-stride).
constexpr int kStepK = 4, kStepChunk = 256 * kStepK;
__global__ void __launch_bounds__(256)
k_dot_partial(int n, const double *__restrict__ a, const double *__restrict__ b, double *__restrict__ partials,
              const PcgCtl *ctl)
{
   if (ctl && ctl->done) { return; }  // (wave-uniform)
   double s = 0.0;
   const long n2 = n / 2, base = (long)blockIdx.x * kStepChunk + threadIdx.x;
   const v2d *a2 = reinterpret_cast<const v2d *>(a), *b2 = reinterpret_cast<const v2d *>(b);
#pragma unroll
   for (int k = 0; k < kStepK; k++)
   {
      const long i = base + 256 * k;
      if (i < n2)
      {
         const v2d u = a2[i], v = b2[i];
         s += u.x * v.x;
         s += u.y * v.y;
      }
   }
   if ((n & 1) && blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) { s += a[n - 1] * b[n - 1]; }
   dot_park(s, partials);
}

// pass 2 (one workgroup of kFinalThreads): the partials in a fixed order; optionally a stopping test on
// the result.  (1,024 threads: the 4,921 energy partials of a C4 Mult are 5 loads per thread, not 20 --
// a latency-bound single workgroup, 8.5 -> ~4 us per PCG iteration, profiles/r6/gpu3.)
constexpr int kFinalThreads = 1024;
__global__ void __launch_bounds__(kFinalThreads)
k_dot_final(int nparts, const double *__restrict__ partials, double *__restrict__ out, double *__restrict__ hout,
            const PcgCtl *ctl, PcgCheck chk, int with_check)
{
   if (ctl && ctl->done) { return; }
   constexpr int NW = kFinalThreads / 64, U = 8;
   __shared__ double red[NW];
   // eight loads in flight per thread (a fixed order: eight running sums, then their pairwise sum), for
   // long partial lists: one partial per brick (78,608 at C5) took 77 dependent loads per thread
   double a[U] = {};
   int i = threadIdx.x;
   for (; i + (U - 1) * kFinalThreads < nparts; i += U * kFinalThreads)
   {
#pragma unroll
      for (int u = 0; u < U; u++) { a[u] += partials[i + u * kFinalThreads]; }
   }
   for (; i < nparts; i += kFinalThreads) { a[0] += partials[i]; }
   double s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   if (threadIdx.x == 0)
   {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < NW; k += 2) { v += red[k] + red[k + 1]; }
      *out = v;
      if (hout) { *hout = v; }  // mapped pinned host mirror (the solver's read-back)
      if (with_check) { pcg_check_one(v, chk); }
   }
}

// The residual half of CGSolver's update (solvers.cpp:930-947): alpha = nom/den; r -= alpha A d;
// z = dinv .* r (jacobi) and the partial sums of r.z (or r.r), one per workgroup in a fixed order,
// finished by k_dot_final.  z holds A d on entry; z is not stored (k_pcg_update_xd forms it again from
// r where it is consumed: 4 vector streams here instead of 8).  x += alpha d is deferred to
// k_pcg_update_xd (or k_pcg_finish_x after the stop), which reads d anyway.  Same arithmetic per entry
// as CGSolver's add / Mult(prec) / Dot.  alpha_out: alpha of the last step run.  16-byte accesses, a
// grid-stride loop over kStepBlocks workgroups.  (The flat chunked grid of k_dot_partial was tried here
// too: a GPU test later in the same process aborted in garbage collection with it, reproducibly, and
// passed with this form -- profiles/r6/gpu5-gpu9; not diagnosed further, so this form stays.)
constexpr int kStepBlocks = 1024;
__global__ void __launch_bounds__(256)
k_pcg_step_r(int n, const double *__restrict__ nom, const double *__restrict__ den, const double *__restrict__ z,
             double *__restrict__ r, const double *__restrict__ dinv, double *__restrict__ partials,
             double *__restrict__ alpha_out, const PcgCtl *ctl)
{
   if (ctl && ctl->done) { return; }
   const double alpha = *nom / *den;
   if (blockIdx.x == 0 && threadIdx.x == 0) { *alpha_out = alpha; }
   double s = 0.0;
   const long n2 = n / 2, stride = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   const v2d *z2 = reinterpret_cast<const v2d *>(z), *q2 = reinterpret_cast<const v2d *>(dinv);
   v2d *r2 = reinterpret_cast<v2d *>(r);
   for (long i = t; i < n2; i += stride)
   {
      const v2d rn = r2[i] + (-alpha) * z2[i];
      r2[i] = rn;
      if (dinv)
      {
         const v2d q = q2[i];
         s += rn.x * (q.x * rn.x);
         s += rn.y * (q.y * rn.y);
      }
      else
      {
         s += rn.x * rn.x;
         s += rn.y * rn.y;
      }
   }
   if ((n & 1) && t == stride - 1)  // the odd tail
   {
      const long i = n - 1;
      const double rn = r[i] + (-alpha) * z[i];
      r[i] = rn;
      s += dinv ? rn * (dinv[i] * rn) : rn * rn;
   }
   dot_park(s, partials);
}

// The direction half (solvers.cpp:930, 985-990): x += alpha d (this iteration's alpha = nom/den,
// deferred from k_pcg_step_r), then d = z + (betanom/nom) d with z = dinv .* r formed here.
// 6 vector streams (x, d, r, dinv read; x, d written) instead of k_pcg_step's x part and
// k_pcg_update_d's 3 + the stored z.
__global__ void __launch_bounds__(256)
k_pcg_update_xd(int n, const double *__restrict__ nom, const double *__restrict__ den,
                const double *__restrict__ betanom, double *__restrict__ x, double *__restrict__ d,
                const double *__restrict__ r, const double *__restrict__ dinv, const PcgCtl *ctl)
{
   // 16-byte accesses: entries 2i, 2i + 1 per lane (the last lane of an odd n takes the tail)
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x, n2 = n / 2;
   if (i > n2 || (ctl && ctl->done)) { return; }
   const double alpha = *nom / *den, beta = *betanom / *nom;
   if (i < n2)
   {
      v2d *x2 = reinterpret_cast<v2d *>(x), *d2 = reinterpret_cast<v2d *>(d);
      const v2d *r2 = reinterpret_cast<const v2d *>(r), *q2 = reinterpret_cast<const v2d *>(dinv);
      const v2d dold = d2[i];
      x2[i] = x2[i] + alpha * dold;
      const v2d z = dinv ? q2[i] * r2[i] : r2[i];
      d2[i] = z + beta * dold;
   }
   else if (n & 1)
   {
      const long j = n - 1;
      const double dold = d[j];
      x[j] = x[j] + alpha * dold;
      const double z = dinv ? dinv[j] * r[j] : r[j];
      d[j] = z + beta * dold;
   }
}

// After the loop: the stopping iteration's x += alpha d, when the stop came from its betanom test
// (converged, max_iter, (B r, r) < 0: CGSolver has already added alpha d then); a den == 0 stop
// comes after k_pcg_update_xd has run (x complete).
__global__ void k_pcg_finish_x(int n, const double *__restrict__ alpha, const double *__restrict__ d,
                               double *__restrict__ x, const PcgCtl *ctl)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   const int done = ctl->done;
   if (i >= n || !(done == PCG_CONVERGED || done == PCG_MAX_ITER || done == PCG_NEG_BR)) { return; }
   x[i] = x[i] + *alpha * d[i];
}

// ConstrainedOperator around a Mult without a vector copy: saved = v[ess], v[ess] = 0 ...
__global__ void k_ess_save_zero(int n, const int *__restrict__ idx, double *__restrict__ v,
                                double *__restrict__ saved)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { saved[i] = v[idx[i]]; v[idx[i]] = 0.0; }
}

// ... then v[ess] = y[ess] = saved (DIAG_ONE rows); sq_parts (optional): the block's sum of saved^2,
// the ess rows' part of (A v, v) = (A v~, v~) + sum_ess v^2 with v~ = v, ess zeroed
__global__ void __launch_bounds__(256)
k_ess_restore(int n, const int *__restrict__ idx, const double *__restrict__ saved, double *__restrict__ v,
              double *__restrict__ y, double *__restrict__ sq_parts)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   double sq = 0.0;
   if (i < n)
   {
      const double sv = saved[i];
      v[idx[i]] = sv;
      y[idx[i]] = sv;
      sq = sv * sv;
   }
   if (sq_parts) { dot_park(sq, sq_parts); }
}

__global__ void k_pcg_precond(int n, const double *__restrict__ dinv, const double *__restrict__ r,
                              double *__restrict__ z)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { z[i] = dinv ? dinv[i] * r[i] : r[i]; }
}

// one thread: a stopping test after a distributed dot's all-reduce
__global__ void k_pcg_check(const double *__restrict__ v, PcgCheck chk) { pcg_check_one(*v, chk); }

__global__ void k_scale(int n, double a, double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[i] *= a; }
}

// out = x + c k  (out may alias x)
__global__ void k_add_scaled(int n, const double *x, double c, const double *__restrict__ k, double *out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = x[i] + c * k[i]; }
}

// STREAM copy (measurement only): 16-byte nontemporal loads and stores, grid-stride,
// the access shape of the guide's 6.29 TB/s float4-copy figure.
// STREAM copy for the roofline reference: 16-byte nontemporal accesses, four independent
// loads in flight per thread before their stores (one in flight per thread measured ~5.4 TB/s).
// HBM copy peak (bench.py's stream_copy_gbs): one 16-byte nontemporal load and store per thread, a flat
// grid -- the fastest form of profiles/calib/copy_probe.hip (6.67 TB/s; the grid-stride form this
// replaces read 4.6-5.4 TB/s, profiles/r6/copy_probe.json).
__global__ void __launch_bounds__(256) k_stream_copy(long n2, const v2d *__restrict__ a, v2d *__restrict__ b)
{
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n2) { __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i); }
}

// Read-only stream: one 16-byte nontemporal load per thread per step, 8 workgroups of 256
// per CU (profiles/calib/read_probe.hip: the fastest of the probed depths and grids, ~7 TB/s;
// deeper per-thread unrolling reads slower).
__global__ void __launch_bounds__(256) k_stream_read(long n2, const v2d *__restrict__ a, double *__restrict__ out)
{
   const long stride = (long)gridDim.x * blockDim.x;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   v2d acc = {0.0, 0.0};
   for (long i = t; i < n2; i += stride) { acc += __builtin_nontemporal_load(a + i); }
   out[t] = acc.x + acc.y;
}

__global__ void k_reciprocal(int n, const double *__restrict__ a, double *__restrict__ out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = 1.0 / a[i]; }
}

__global__ void k_gather_idx(int n, const int *__restrict__ idx, const double *__restrict__ x,
                             double *__restrict__ buf)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { buf[i] = x[idx[i]]; }
}

__global__ void k_scatter_add_idx(int n, const int *__restrict__ idx, const double *__restrict__ buf,
                                  double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   // atomic: a dof shared by >= 3 ranks appears in several neighbour segments
   if (i < n) { unsafeAtomicAdd(y + idx[i], buf[i]); }
}

// Second pass of the deterministic scatter, run-compressed (pa_form.cpp, build_shared_plan):
// the shared dofs of a brick face or a lane row form runs -- 1D or 2D lattices of plan
// entries whose dof and every holder's partial slot are affine in the entry's position.  A
// workgroup takes whole runs (<= 256 entries), stages their 48-byte descriptors in LDS in one
// coalesced read, and each thread finds its run there: two dependent global reads before the
// partials (block table, descriptors), as the per-entry plan had (meta, slot list), with ~12
// instead of ~24 plan bytes per 2-holder dof.  A dof's holders are summed in ascending slot
// order.  Workgroups are taken in XCD-contiguous order (neighbouring runs, neighbouring slots).
constexpr int kRunInts = 12;
__global__ void __launch_bounds__(256)
k_sum_partials(int b0, int b1, const int *__restrict__ blocks, const int *__restrict__ runs,
               const int *__restrict__ rslots, const int *__restrict__ pdof, const double *__restrict__ part,
               int n_owned, double *__restrict__ y, double *__restrict__ yg)
{
   __shared__ int sd[257 * kRunInts];
   const int blk = b0 + xcd_contiguous(blockIdx.x, gridDim.x);
   if (blk >= b1) { return; }  // whole workgroup
   // block row: first run, end run, first entry, entries | explicit-dof runs << 30 (scalar loads)
   const int r0 = blocks[4 * blk], nr = blocks[4 * blk + 1] - r0, e0 = blocks[4 * blk + 2], bn = blocks[4 * blk + 3];
   const int i = e0 + (int)threadIdx.x;
   const bool live = (int)threadIdx.x < (bn & 0xffff);
   // a block with explicit-dof runs issues its entries' dofs now, beside the descriptor staging
   // (the entry list holds every entry's dof), instead of after the run lookup
   const int dpre = ((bn >> 30) & 1) && live ? pdof[i] : 0;
   for (int k = threadIdx.x; k < (nr + 1) * kRunInts; k += blockDim.x) { sd[k] = runs[(size_t)r0 * kRunInts + k]; }
   __syncthreads();
   if (!live) { return; }
   int lo = 0, hi = nr - 1;
   while (lo < hi)
   {
      const int mid = (lo + hi + 1) >> 1;
      if (sd[mid * kRunInts + 6] <= i) { lo = mid; }
      else { hi = mid - 1; }
   }
   const int *R = sd + lo * kRunInts;
   const int shape = R[0], n1 = shape & 255, cnt = (shape >> 16) & 255;
   const int off = i - R[6], pa = off % n1, pb = off / n1;
   // shape bit 24: the run's dofs are not a lattice (entity numbering): the entry list holds them
   const int d = (shape >> 24) ? dpre : R[1] + pa * R[2] + pb * R[3];
   const int ds = pa * R[4] + pb * R[5];
   double v[4];
#pragma unroll
   for (int k = 0; k < 4; k++) { v[k] = k < cnt ? part[R[8 + k] + ds] : 0.0; }
   double acc = 0.0;
#pragma unroll
   for (int k = 0; k < 4; k++) { acc += v[k]; }
   for (int k = 4; k < cnt; k++) { acc += part[rslots[R[7] + k] + ds]; }
   if (d < n_owned) { y[d] = acc; }
   else { yg[d - n_owned] = acc; }
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_wpe_mdq(const ApplyArgs &a, bool in_e, bool out_e, const Basis1D &b, hipStream_t s)
{
   constexpr int NQ = Q * Q * Q;
   const int nt = ((NQ + 63) / 64) * 64;
   const int e0 = a.blk_begin * 64, e1 = std::min(a.ne, a.blk_end * 64);
   if (e1 <= e0) { return; }
   hipLaunchKernelGGL((k_apply_wpe<D, Q, MASS, DIFF>), dim3(e1 - e0), dim3(nt), 0, s, a.pos, a.kind, a.ne, e0,
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, in_e, out_e);
}

template <int D, int Q>
void launch_wpe_dq(bool mass, bool diff, const ApplyArgs &a, bool in_e, bool out_e,
                   const Basis1D &b, hipStream_t s)
{
   if (mass && diff) { launch_wpe_mdq<D, Q, true, true>(a, in_e, out_e, b, s); }
   else if (mass) { launch_wpe_mdq<D, Q, true, false>(a, in_e, out_e, b, s); }
   else if (diff) { launch_wpe_mdq<D, Q, false, true>(a, in_e, out_e, b, s); }
}

} // namespace

namespace kern
{

void apply_wpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, bool in_e, bool out_e,
               const Basis1D &b, hipStream_t s)
{
   if (a.ne == 0) { return; }
#define ECM2_WPE_CASE(DD, QQ)                                         \
   if (D == DD && Q == QQ)                                            \
   {                                                                  \
      launch_wpe_dq<DD, QQ>(mass, diff, a, in_e, out_e, b, s);        \
      ECM2_HIP(hipGetLastError());                                    \
      return;                                                         \
   }
   ECM2_WPE_CASE(2, 3)
   ECM2_WPE_CASE(3, 4)
   ECM2_WPE_CASE(4, 5)
   ECM2_WPE_CASE(5, 6)
   ECM2_WPE_CASE(2, 2)
   ECM2_WPE_CASE(3, 3)
   ECM2_WPE_CASE(4, 4)
   ECM2_WPE_CASE(5, 5)
   ECM2_WPE_CASE(6, 7)
   // Q1D = D1D + 2: the rule a quadratic mesh's MassIntegrator asks for (GetRule adds Trans.OrderW(),
   // bilininteg.cpp:1450-1462), or a user rule (IntRule)
   ECM2_WPE_CASE(2, 4)
   ECM2_WPE_CASE(3, 5)
   ECM2_WPE_CASE(4, 6)
   ECM2_WPE_CASE(5, 7)
   ECM2_WPE_CASE(6, 8)
#undef ECM2_WPE_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "no PA kernel for D1D=" << D << " Q1D=" << Q);
}

void restriction_mult(long n, int nd, const int *gm, const double *x, double *xe, hipStream_t s)
{
   (void)nd;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_restriction_mult, dim3(grid_for(n, 256)), dim3(256), 0, s, n, gm, x, xe);
   ECM2_HIP(hipGetLastError());
}

void restriction_mult_transpose(int ndofs, int nd, const int *offsets, const int *indices,
                                const double *xe, double *y, hipStream_t s)
{
   (void)nd;
   if (ndofs == 0) { return; }
   hipLaunchKernelGGL(k_restriction_mult_transpose, dim3(grid_for(ndofs, 256)), dim3(256), 0, s,
                      ndofs, offsets, indices, xe, y);
   ECM2_HIP(hipGetLastError());
}

void diagonal_generic(const int *pos, int D, int Q, int layout, int ne, const int *gm, const double *qdd,
                      const double *qdm, double *diag, bool out_e, const Basis1D &b, hipStream_t s)
{
   const long n = (long)ne * D * D * D;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_diagonal, dim3(grid_for(n, 128)), dim3(128), 0, s, pos, D, Q, layout, ne, gm,
                      qdd, qdm, diag, out_e, b);
   ECM2_HIP(hipGetLastError());
}

void set_values(int n, const int *idx, double val, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_set_values, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, val, y);
   ECM2_HIP(hipGetLastError());
}

void copy_values(int n, const int *idx, const double *x, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_copy_values, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, x, y);
   ECM2_HIP(hipGetLastError());
}

int step_parts(int n) { return std::max(1, (int)((n / 2 + kStepChunk - 1) / kStepChunk)); }

static PcgCheck to_check(const PcgStop *stop)
{
   return stop ? PcgCheck{stop->r0, stop->it, stop->max_iter, stop->ctl, stop->host, stop->betanom, stop->kind}
               : PcgCheck{};
}

void dot(int n, const double *a, const double *b, double *partials, double *out, hipStream_t s, double *hout,
         const PcgCtl *ctl, const PcgStop *stop)
{
   const int nb = step_parts(n);
   hipLaunchKernelGGL(k_dot_partial, dim3(nb), dim3(256), 0, s, n, a, b, partials, ctl);
   hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(kFinalThreads), 0, s, nb, partials, out, hout, ctl, to_check(stop),
                      stop ? 1 : 0);
   ECM2_HIP(hipGetLastError());
}

void pcg_step_r(int n, const double *nom, const double *den, const double *z, double *r, const double *dinv,
                double *partials, double *out, double *alpha, hipStream_t s, const PcgCtl *ctl, const PcgStop *stop)
{
   const int nb = kStepBlocks;
   hipLaunchKernelGGL(k_pcg_step_r, dim3(nb), dim3(256), 0, s, n, nom, den, z, r, dinv, partials, alpha, ctl);
   hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(kFinalThreads), 0, s, nb, partials, out, nullptr, ctl, to_check(stop),
                      stop ? 1 : 0);
   ECM2_HIP(hipGetLastError());
}

void pcg_update_xd(int n, const double *nom, const double *den, const double *betanom, double *x, double *d,
                   const double *r, const double *dinv, hipStream_t s, const PcgCtl *ctl)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_pcg_update_xd, dim3(grid_for(n / 2 + 1, 256)), dim3(256), 0, s, n, nom, den, betanom, x, d,
                      r, dinv, ctl);
   ECM2_HIP(hipGetLastError());
}

void pcg_finish_x(int n, const double *alpha, const double *d, double *x, hipStream_t s, const PcgCtl *ctl)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_pcg_finish_x, dim3(grid_for(n, 256)), dim3(256), 0, s, n, alpha, d, x, ctl);
   ECM2_HIP(hipGetLastError());
}

void pcg_check(const double *v, const PcgStop &stop, hipStream_t s)
{
   hipLaunchKernelGGL(k_pcg_check, dim3(1), dim3(1), 0, s, v, to_check(&stop));
   ECM2_HIP(hipGetLastError());
}

void ess_save_zero(int n, const int *idx, double *v, double *saved, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_ess_save_zero, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, v, saved);
   ECM2_HIP(hipGetLastError());
}

void ess_restore(int n, const int *idx, const double *saved, double *v, double *y, hipStream_t s, double *sq_parts)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_ess_restore, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, saved, v, y, sq_parts);
   ECM2_HIP(hipGetLastError());
}

int ess_parts(int n) { return n > 0 ? grid_for(n, 256) : 0; }

void dot_final(int nparts, const double *partials, double *out, hipStream_t s, const PcgCtl *ctl,
               const PcgStop *stop, double *hout)
{
   hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(kFinalThreads), 0, s, nparts, partials, out, hout, ctl, to_check(stop),
                      stop ? 1 : 0);
   ECM2_HIP(hipGetLastError());
}

void pcg_precond(int n, const double *dinv, const double *r, double *z, hipStream_t s)
{
   hipLaunchKernelGGL(k_pcg_precond, dim3(grid_for(n, 256)), dim3(256), 0, s, n, dinv, r, z);
   ECM2_HIP(hipGetLastError());
}

void scale(int n, double a, double *y, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_scale, dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, y);
   ECM2_HIP(hipGetLastError());
}

void add_scaled(int n, const double *x, double c, const double *k, double *out, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_add_scaled, dim3(grid_for(n, 256)), dim3(256), 0, s, n, x, c, k, out);
   ECM2_HIP(hipGetLastError());
}

void stream_copy(long n, const double *a, double *b, hipStream_t s)
{
   ECM2_VERIFY(n % 2 == 0 && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0, ERR_ARG,
               "stream_copy needs 16-byte aligned even-length arrays");
   const long n2 = n / 2;
   hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, s, n2,
                      reinterpret_cast<const v2d *>(a), reinterpret_cast<v2d *>(b));
   ECM2_HIP(hipGetLastError());
}

void stream_read(long n, const double *a, double *out, long nout, hipStream_t s)
{
   static int cus = 0;
   if (!cus)
   {
      int dev = 0;
      ECM2_HIP(hipGetDevice(&dev));
      ECM2_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
   }
   const long blocks = 8L * cus, threads = blocks * 256;
   ECM2_VERIFY(nout >= threads, ERR_ARG, "stream_read needs " << threads << " outputs");
   hipLaunchKernelGGL(k_stream_read, dim3(blocks), dim3(256), 0, s, n / 2, reinterpret_cast<const v2d *>(a), out);
   ECM2_HIP(hipGetLastError());
}

void reciprocal(int n, const double *a, double *out, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_reciprocal, dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, out);
   ECM2_HIP(hipGetLastError());
}

void gather_idx(int n, const int *idx, const double *x, double *buf, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_gather_idx, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, x, buf);
   ECM2_HIP(hipGetLastError());
}

void scatter_add_idx(int n, const int *idx, const double *buf, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_scatter_add_idx, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, buf, y);
   ECM2_HIP(hipGetLastError());
}

void sum_partials(int b0, int b1, const int *blocks, const int *runs, const int *rslots, const int *pdof,
                  const double *part, int n_owned, double *y, double *yg, hipStream_t s)
{
   if (b1 <= b0) { return; }
   ECM2_VERIFY(blocks && runs && pdof, ERR_INTERNAL, "summation pass needs its run plan");
   hipLaunchKernelGGL(k_sum_partials, dim3(b1 - b0), dim3(256), 0, s, b0, b1, blocks, runs, rslots, pdof, part,
                      n_owned, y, yg);
   ECM2_HIP(hipGetLastError());
}

} // namespace kern
} // namespace ecm2
