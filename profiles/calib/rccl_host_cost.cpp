// Host cost of one grouped RCCL point-to-point exchange as the serial distributed Mult issues it
// (ncclGroupStart, 2 x ncclSend + 2 x ncclRecv of one dof plane each, ncclGroupEnd), on a one-rank
// communicator (sends to itself): microseconds of host time per exchange when enqueued back to back,
// and the GPU time per exchange after a final synchronize.  Build: see profiles/rccl_host_cost.sh.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { auto r_ = (x); if (r_ != 0) { std::printf("error %d at %s\n", (int)r_, #x); return 1; } } while (0)

int main()
{
   const int n = 47089;  // one 217 x 217 dof plane (C4 z-slabs), 377 KB
   ncclUniqueId id;
   CK(ncclGetUniqueId(&id));
   ncclComm_t comm;
   CK(ncclCommInitRank(&comm, 1, id, 0));
   hipStream_t st;
   CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
   double *a, *b;
   CK(hipMalloc(&a, 4 * n * sizeof(double)));
   CK(hipMalloc(&b, 4 * n * sizeof(double)));
   auto exchange = [&]() -> int {
      CK(ncclGroupStart());
      CK(ncclSend(a, n, ncclFloat64, 0, comm, st));
      CK(ncclSend(a + n, n, ncclFloat64, 0, comm, st));
      CK(ncclRecv(b, n, ncclFloat64, 0, comm, st));
      CK(ncclRecv(b + n, n, ncclFloat64, 0, comm, st));
      CK(ncclGroupEnd());
      return 0;
   };
   for (int i = 0; i < 50; i++) { if (exchange()) { return 1; } }
   CK(hipStreamSynchronize(st));
   for (int rep = 0; rep < 3; rep++)
   {
      const int iters = 500;
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; i++) { if (exchange()) { return 1; } }
      auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(st));
      auto t2 = std::chrono::steady_clock::now();
      const double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
      const double all = std::chrono::duration<double, std::micro>(t2 - t0).count() / iters;
      std::printf("grouped 2x(send+recv) of %d doubles: host %.2f us per exchange, host+GPU %.2f us per exchange\n",
                  n, host, all);
   }
   (void)hipFree(a);
   (void)hipFree(b);
   (void)ncclCommDestroy(comm);
   (void)hipStreamDestroy(st);
   return 0;
}
