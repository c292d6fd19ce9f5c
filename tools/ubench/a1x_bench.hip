// Microbenchmark of the scan kernel's A1 step variants in isolation (8 waves
// per block, 1 block per CU, 256 blocks): s_memtime ticks and ns per query.
//   exact : sequential sub/mul/add distances + a1_reduce (the exact path)
//   fma2  : expanded-form bounds, two queries per trip (the batch path)
//   fmaonly / exactonly : distances + in-lane min only (the floors)
#include "../../soundchunks_amd/csrc/gsc_scan.hip"
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
// packed: leaves (2i, 2i+1) of a lane in one 64-bit register pair
__device__ __forceinline__ void a1_dist_pk2(const f2 (&c2)[4][16], const float (&cn)[8], const float* __restrict__ qm0,
                                            const float* __restrict__ qm1, float (&dv0)[8], float (&dv1)[8]) {
    f2 a0[4], a1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a0[i] = f2{cn[2 * i], cn[2 * i + 1]};
        a1[i] = a0[i];
    }
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        const f2 m0 = f2{qm0[d], qm0[d]}, m1 = f2{qm1[d], qm1[d]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a0[i] = __builtin_elementwise_fma(m0, c2[i][d], a0[i]);
            a1[i] = __builtin_elementwise_fma(m1, c2[i][d], a1[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dv0[2 * i] = a0[i].x;
        dv0[2 * i + 1] = a0[i].y;
        dv1[2 * i] = a1[i].x;
        dv1[2 * i + 1] = a1[i].y;
    }
}

template <int MODE>
__global__ __launch_bounds__(512) void a1k(const float* __restrict__ in, float* __restrict__ out, int batches,
                                           unsigned long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Scan2Shared& sh = *reinterpret_cast<Scan2Shared*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 2 * kBatch * 16; i += blockDim.x) {
        (&sh.q[0][0][0])[i] = in[i];
        (&sh.qm[0][0][0])[i] = -2.0f * in[i];
    }
    float creg[8][16], cn[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int d = 0; d < 16; ++d) creg[s][d] = in[((tid * 8 + s) & 255) * 16 + d];
        cn[s] = norm2_x<16>(creg[s]);
    }
    f2 c2[4][16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int d = 0; d < 16; ++d) c2[i][d] = f2{creg[2 * i][d], creg[2 * i + 1][d]};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll 1
    for (int b = 0; b < batches; ++b) {
        const int buf = b & 1;
#pragma unroll 1
        for (int jj = 0; jj < kBatch; jj += 2) {
            float dv0[8], dv1[8];
            if (MODE == 0 || MODE == 3) {
                a1_dist<16>(creg, sh.q[buf][jj], dv0);
                a1_dist<16>(creg, sh.q[buf][jj + 1], dv1);
            } else if (MODE == 4 || MODE == 5 || MODE == 7) {
                a1_dist_pk2(c2, cn, sh.qm[buf][jj], sh.qm[buf][jj + 1], dv0, dv1);
            } else {
                a1_dist_x2<16>(creg, cn, sh.qm[buf][jj], sh.qm[buf][jj + 1], dv0, dv1);
            }
            if (MODE <= 1 || MODE == 5) {
                a1_reduce<12>(dv0, sh.wrec[wave][jj], wave, lane);
                a1_reduce<12>(dv1, sh.wrec[wave][jj + 1], wave, lane);
            } else if (MODE >= 6) {
                a1_reduce2<12>(dv0, dv1, sh.wrec[wave][jj], sh.wrec[wave][jj + 1], wave, lane);
            } else {
                float m = dv0[0];
#pragma unroll
                for (int s = 1; s < 8; ++s) m = fminf(m, dv0[s]);
#pragma unroll
                for (int s = 0; s < 8; ++s) m = fminf(m, dv1[s]);
                acc ^= __float_as_uint(m);
            }
        }
        __syncthreads();
        if ((MODE <= 1 || MODE >= 5) && lane == 0) acc ^= sh.wrec[wave][b & 31].minbits ^ sh.wrec[wave][b & 31].sl[5];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = __uint_as_float(acc);
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, float* din, float* dout, unsigned long long* dc, int nblk) {
    const int batches = 400;
    const size_t shm = sizeof(Scan2Shared);
    hipFuncSetAttribute((const void*)a1k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL((a1k<MODE>), dim3(nblk), dim3(512), shm, 0, din, dout, batches, dc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((a1k<MODE>), dim3(nblk), dim3(512), shm, 0, din, dout, batches, dc);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c0;
    hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost);
    const double q = (double)batches * kBatch;
    printf("%-10s blocks %3d  %7.1f ticks/query  %7.1f ns/query  (tick rate %.0f MHz)\n", name, nblk, (double)c0 / q,
           ms * 1e6 / q, (double)c0 / (ms * 1e3));
}

int main() {
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 8192 * 4);
    hipMalloc(&dout, 1 << 22);
    hipMalloc(&dc, 8 * 512);
    static float h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (float)((i * 37) % 101) * 0.01f;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nb : {1, 256}) {
        run<0>("exact", din, dout, dc, nb);
        run<1>("fma2", din, dout, dc, nb);
        run<3>("exactonly", din, dout, dc, nb);
        run<2>("fmaonly", din, dout, dc, nb);
        run<4>("pkonly", din, dout, dc, nb);
        run<5>("pk2", din, dout, dc, nb);
        run<6>("fma_r2", din, dout, dc, nb);
        run<7>("pk_r2", din, dout, dc, nb);
    }
    return 0;
}
