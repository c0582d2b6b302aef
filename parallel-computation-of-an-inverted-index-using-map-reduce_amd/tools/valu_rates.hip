// valu_rates.hip — issue cost of the integer instructions the tokenizer's
// per-token step leans on (v_mul_lo_u32, v_mad_u64_u32, v_mul_u32_u24,
// v_dot4_u32_u8, v_add_u32), measured as a dependent chain per lane across
// the whole GPU: ns per wave-instruction per CU.  Guides the choice of hash
// and packing instructions in ii_kernels.h.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int kIters = 4096;

template <int kOp>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
    uint32_t a = seed ^ threadIdx.x, b = seed * 3u + blockIdx.x, c = 0x9E3779B1u, d = a ^ 0x85EBCA77u;
#pragma unroll 16
    for (int i = 0; i < kIters; i++) {
        // four independent chains per lane, so latency does not hide the rate
        if (kOp == 0) {
            a += c; b += c; d += a; c += b;
        } else if (kOp == 1) {
            a *= b | 1u; b *= d | 1u; d *= c | 1u; c *= a | 1u;
        } else if (kOp == 2) {
            a = __builtin_amdgcn_udot4(a, 0x01200000u, b, false);
            b = __builtin_amdgcn_udot4(b, 0x00000120u, a, false);
            d = __builtin_amdgcn_udot4(d, 0x08040201u, c, false);
            c = __builtin_amdgcn_udot4(c, 0x80402010u, d, false);
        } else if (kOp == 3) {
            a = __umul24(a, 0x9E3779u) + b;
            b = __umul24(b, 0x85EBCAu) + a;
            d = __umul24(d, 0x2C1B3Cu) + c;
            c = __umul24(c, 0x27D4EBu) + d;
        } else {
            const uint64_t p = (uint64_t)a * 0x9E3779B1u + b;
            const uint64_t q = (uint64_t)d * 0x85EBCA77u + c;
            a = (uint32_t)p; b = (uint32_t)(p >> 32); d = (uint32_t)q; c = (uint32_t)(q >> 32);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

template <int kOp>
static int run(const char* name, int ninst, uint32_t* out, int cus) {
    const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    k_rate<kOp><<<blocks, 256>>>(out, 1);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(e0));
        k_rate<kOp><<<blocks, 256>>>(out, (uint32_t)r);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double winst = (double)blocks * 4 * kIters * ninst;  // wave-instructions
    printf("%-28s %8.3f ms  %6.2f ns per wave-instr per CU  (%.2f wave-instr / CU / ns)\n", name, best,
           best * 1e6 / (winst / cus), winst / cus / (best * 1e6));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(uint32_t)));
    printf("%d CUs, %d MHz\n", cus, p.clockRate / 1000);
    if (run<0>("v_add_u32 x4", 4, out, cus)) return 1;
    if (run<1>("(v_or + v_mul_lo_u32) x4", 8, out, cus)) return 1;
    if (run<2>("v_dot4_u32_u8 x4", 4, out, cus)) return 1;
    if (run<3>("v_mul_u32_u24 + add x4", 8, out, cus)) return 1;
    if (run<4>("v_mad_u64_u32 x2", 2, out, cus)) return 1;
    return 0;
}
