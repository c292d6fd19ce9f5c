// Packed f32 (v_pk_add_f32 / v_pk_mul_f32) for the A1 distance loop:
//   1. bit-exactness against scalar v_add/v_sub/v_mul on random bit patterns
//      (normals, denormals, zeros, infinities, NaN payloads aside);
//   2. ticks per query for the 8-leaf x 16-dim distance body, scalar vs packed,
//      8 waves per CU (one block per CU, 256 blocks), s_memtime + hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t rng(uint32_t& s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

__global__ void check(unsigned long long* bad, int iters) {
    uint32_t s = 0x9E3779B9u ^ (blockIdx.x * 1024 + threadIdx.x) * 2654435761u;
    unsigned long long nb = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t ua = rng(s), ub = rng(s), uc = rng(s), ud = rng(s);
        // bias towards small exponents (denormals) a quarter of the time
        if ((ua & 3) == 0) ua &= 0x80FFFFFFu;
        if ((ub & 3) == 1) ub &= 0x80FFFFFFu;
        const float a = __uint_as_float(ua), b = __uint_as_float(ub), c = __uint_as_float(uc), d = __uint_as_float(ud);
        if (a != a || b != b || c != c || d != d) continue;
        f2 x = {a, c}, y = {b, d};
        f2 ps = x + y, pd = x - y, pm = x * y;
        asm volatile("" : "+v"(ps), "+v"(pd), "+v"(pm));
        const float s0 = __fadd_rn(a, b), s1 = __fadd_rn(c, d);
        const float d0 = __fsub_rn(a, b), d1 = __fsub_rn(c, d);
        const float m0 = __fmul_rn(a, b), m1 = __fmul_rn(c, d);
        auto ne = [](float p, float q) { return __float_as_uint(p) != __float_as_uint(q) && !(p != p && q != q); };
        nb += ne(ps.x, s0) + ne(ps.y, s1) + ne(pd.x, d0) + ne(pd.y, d1) + ne(pm.x, m0) + ne(pm.y, m1);
    }
    atomicAdd(bad, nb);
}

template <int D, bool PK>
__global__ __launch_bounds__(512) void dist(const float* __restrict__ in, float* __restrict__ out, int iters,
                                            unsigned long long* cyc) {
    __shared__ float sq[1024 * 16];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024 * D; i += blockDim.x) sq[i] = in[i % 4096];
    __syncthreads();
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (PK) {
        f2 c[4][D];
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int d = 0; d < D; ++d) c[p][d] = f2{in[((tid * 8 + 2 * p) & 255) * D + d], in[((tid * 8 + 2 * p + 1) & 255) * D + d]};
#pragma unroll 1
        for (int it = 0; it < iters; ++it) {
            const float* qv = sq + (it & 1023) * D;
            f2 dv[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) dv[p] = f2{0.0f, 0.0f};
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const f2 q2 = f2{qv[d], qv[d]};
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const f2 t = q2 - c[p][d];
                    dv[p] = dv[p] + t * t;
                }
            }
            uint32_t m = 0xffffffffu;
#pragma unroll
            for (int p = 0; p < 4; ++p) m = min(m, min(__float_as_uint(dv[p].x), __float_as_uint(dv[p].y)));
            acc ^= m;
        }
    } else {
        float c[8][D];
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int d = 0; d < D; ++d) c[s][d] = in[((tid * 8 + s) & 255) * D + d];
#pragma unroll 1
        for (int it = 0; it < iters; ++it) {
            const float* qv = sq + (it & 1023) * D;
            float dv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) dv[s] = 0.0f;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float qd = qv[d];
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const float t = __fsub_rn(qd, c[s][d]);
                    dv[s] = __fadd_rn(dv[s], __fmul_rn(t, t));
                }
            }
            uint32_t m = 0xffffffffu;
#pragma unroll
            for (int s = 0; s < 8; ++s) m = min(m, __float_as_uint(dv[s]));
            acc ^= m;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = __uint_as_float(acc);
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int D, bool PK>
void run(const char* name, float* din, float* dout, unsigned long long* dc, int nblk) {
    const int iters = 20000;
    hipLaunchKernelGGL((dist<D, PK>), dim3(nblk), dim3(512), 0, 0, din, dout, iters, dc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((dist<D, PK>), dim3(nblk), dim3(512), 0, 0, din, dout, iters, dc);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c0;
    hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost);
    // ops per query per CU: 4096 leaves x D x 3
    const double ops = 512.0 * 8 * D * 3 * iters * nblk;
    printf("%-22s blocks %3d  %.1f ticks/query  %.2f Tops/s chip  (tick %.0f MHz)\n", name, nblk, (double)c0 / iters,
           ops / (ms * 1e-3) / 1e12, (double)c0 / (ms * 1e3));
}

int main() {
    unsigned long long* bad;
    hipMalloc(&bad, 8);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, bad, 4096);
    unsigned long long hb = 0;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    printf("packed vs scalar mismatches over %llu op pairs: %llu\n", 1024ull * 256 * 4096 * 3, hb);
    float *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 8192 * 4);
    hipMalloc(&dout, 1 << 22);
    hipMalloc(&dc, 8 * 512);
    static float h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (float)((i * 37) % 101) * 0.01f;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nb : {1, 256}) {
        run<16, false>("scalar D16", din, dout, dc, nb);
        run<16, true>("packed D16", din, dout, dc, nb);
    }
    return 0;
}
