// Issue / dependency microbenchmark for one wave per SIMD (T1 decoder design data): cycles per
// instruction of dependent and independent VALU chains, 64-bit shifts, selects and LDS round trips,
// timed with s_memtime around unrolled inline-asm sequences.  Usage: ./ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP10(x) x x x x x x x x x x
#define REP100(x) REP10(REP10(x))

__global__ void k(unsigned long long* out, uint32_t seed) {
    __shared__ uint32_t lds[64 * 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 64; i += 64) lds[i] = (i + 64) % (64 * 64);   // pointer chase: +64
    __syncthreads();
    uint32_t a = seed + lane, b = seed * 3 + 1, c = lane * 7, d = seed ^ lane, e = 5;
    uint64_t w = ((uint64_t)a << 32) | b;
    unsigned long long t0, t1;
    int slot = 0;
#define TIME(body)                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory"); \
    body;                                                                                          \
    asm volatile("s_waitcnt lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory"); \
    if (lane == 0) out[blockIdx.x * 32 + slot] = t1 - t0;                                          \
    ++slot;
    // 0: 100 dependent v_add_u32
    TIME(asm volatile(REP100("v_add_u32 %0, %0, %1\n") : "+v"(a) : "v"(b)));
    // 1: 100 v_add_u32 in 4 independent chains
    TIME(asm volatile(REP10("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                            "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
                            "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n")
                      : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(b)));
    // 2: 100 dependent v_lshrrev_b64
    TIME(asm volatile(REP100("v_lshrrev_b64 %0, %1, %0\n") : "+v"(w) : "v"(e & 1)));
    // 3: 100 dependent v_cndmask_b32 (vcc mask)
    TIME(asm volatile("v_cmp_gt_u32 vcc, %2, 7\n" REP100("v_cndmask_b32 %0, %1, %0, vcc\n") : "+v"(a) : "v"(c), "v"(d) : "vcc"));
    // 4: 100 dependent v_cndmask_b32_e64 with an SGPR-pair mask from v_cmp (alternating)
    TIME(asm volatile(REP100("v_cmp_lt_u32_e64 s[40:41], %0, %2\n v_cndmask_b32_e64 %0, %1, %0, s[40:41]\n")
                      : "+v"(a) : "v"(c), "v"(d) : "s40", "s41"));
    // 5: 20 dependent ds_read_b32 (pointer chase)
    {
        uint32_t p = lane * 4;
        TIME(asm volatile(REP10("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)\n ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)\n") : "+v"(p)::"memory"));
        a += p;
    }
    // 6: 20 x (ds_or_b32 then dependent ds_read_b32 of the same word)
    {
        uint32_t p = lane * 4, v = 0;
        TIME(asm volatile(REP10("ds_or_b32 %0, %2\n ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n ds_or_b32 %0, %2\n ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n")
                          : "+v"(p), "+v"(v) : "v"(e) : "memory"));
        a += v;
    }
    // 7: 100 SALU s_add_u32 dependent
    {
        uint32_t s = seed;
        TIME(asm volatile(REP100("s_add_u32 %0, %0, 3\n") : "+s"(s)::"scc"));
        a += s;
    }
    // 8: 100 alternating VALU (independent) + SALU
    {
        uint32_t s = seed;
        TIME(asm volatile(REP10("v_add_u32 %0, %0, %2\n s_add_u32 %1, %1, 3\n v_add_u32 %3, %3, %2\n s_add_u32 %1, %1, 3\n v_add_u32 %0, %0, %2\n"
                                "s_add_u32 %1, %1, 3\n v_add_u32 %3, %3, %2\n s_add_u32 %1, %1, 3\n v_add_u32 %0, %0, %2\n s_add_u32 %1, %1, 3\n")
                          : "+v"(a), "+s"(s), "+v"(b), "+v"(c)::"scc"));
        a += s;
    }
    // 9: ds_read2st64_b32 x 6 independent then one wait (throughput + latency)
    {
        uint32_t p = lane * 4; uint64_t r0, r1, r2, r3, r4, r5;
        TIME(asm volatile("ds_read2st64_b32 %0, %6 offset0:1 offset1:2\n ds_read2st64_b32 %1, %6 offset0:3 offset1:4\n"
                          "ds_read2st64_b32 %2, %6 offset0:5 offset1:6\n ds_read2st64_b32 %3, %6 offset0:7 offset1:8\n"
                          "ds_read2st64_b32 %4, %6 offset0:9 offset1:10\n ds_read2st64_b32 %5, %6 offset0:11 offset1:12\n"
                          "s_waitcnt lgkmcnt(0)\n"
                          : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3), "=v"(r4), "=v"(r5)
                          : "v"(p) : "memory"));
        a += (uint32_t)(r0 + r1 + r2 + r3 + r4 + r5);
    }
    // 10: 20 ds_or_b32 (no return) to this lane's words, then one wait
    {
        uint32_t p = lane * 4;
        TIME(asm volatile(REP10("ds_or_b32 %0, %1 offset:256\n ds_or_b32 %0, %1 offset:512\n") "s_waitcnt lgkmcnt(0)\n" : : "v"(p), "v"(e) : "memory"));
    }
    // 11: 20 ds_write_b32 to this lane's words, then one wait
    {
        uint32_t p = lane * 4;
        TIME(asm volatile(REP10("ds_write_b32 %0, %1 offset:256\n ds_write_b32 %0, %1 offset:512\n") "s_waitcnt lgkmcnt(0)\n" : : "v"(p), "v"(e) : "memory"));
    }
    // 12: 10 x (4 ds_or + dependent ds_read)
    {
        uint32_t p = lane * 4, v = 0;
        TIME(asm volatile(REP10("ds_or_b32 %0, %2 offset:256\n ds_or_b32 %0, %2 offset:512\n ds_or_b32 %0, %2 offset:768\n ds_or_b32 %0, %2 offset:1024\n ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n")
                          : "+v"(p), "+v"(v) : "v"(e) : "memory"));
        a += v;
    }
    // 13: 10 x (4 ds_write + dependent ds_read)
    {
        uint32_t p = lane * 4, v = 0;
        TIME(asm volatile(REP10("ds_write_b32 %0, %2 offset:256\n ds_write_b32 %0, %2 offset:512\n ds_write_b32 %0, %2 offset:768\n ds_write_b32 %0, %2 offset:1024\n ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n")
                          : "+v"(p), "+v"(v) : "v"(e) : "memory"));
        a += v;
    }
    // 14: 100 dependent v_cndmask_b32_e64 with a fixed SGPR-pair mask
    TIME(asm volatile("v_cmp_gt_u32_e64 s[40:41], %2, 7\n" REP100("v_cndmask_b32_e64 %0, %1, %0, s[40:41]\n") : "+v"(a) : "v"(c), "v"(d) : "s40", "s41"));
    // 15: 20 x (s_cmp + taken s_cbranch_scc1 to the next instruction + v_add)
    {
        uint32_t s = seed;
        TIME(asm volatile(REP10("s_cmp_eq_u32 %1, %1\n s_cbranch_scc1 1f\n v_add_u32 %0, %0, %2\n1:\n v_add_u32 %0, %0, %2\n"
                                "s_cmp_eq_u32 %1, %1\n s_cbranch_scc1 2f\n v_add_u32 %0, %0, %2\n2:\n v_add_u32 %0, %0, %2\n")
                          : "+v"(a) : "s"(s), "v"(b) : "scc"));
    }
    // 16: 20 x (s_cmp + not-taken s_cbranch_scc0 + v_add + v_add)
    {
        uint32_t s = seed;
        TIME(asm volatile(REP10("s_cmp_eq_u32 %1, %1\n s_cbranch_scc0 1f\n v_add_u32 %0, %0, %2\n1:\n v_add_u32 %0, %0, %2\n"
                                "s_cmp_eq_u32 %1, %1\n s_cbranch_scc0 2f\n v_add_u32 %0, %0, %2\n2:\n v_add_u32 %0, %0, %2\n")
                          : "+v"(a) : "s"(s), "v"(b) : "scc"));
    }
    // 17: 20 x (v_cmp -> vcc, s_cbranch_vccz taken, v_add)
    {
        TIME(asm volatile(REP10("v_cmp_gt_u32 vcc, %1, %1\n s_cbranch_vccz 1f\n v_add_u32 %0, %0, %1\n1:\n v_add_u32 %0, %0, %1\n"
                                "v_cmp_gt_u32 vcc, %1, %1\n s_cbranch_vccz 2f\n v_add_u32 %0, %0, %1\n2:\n v_add_u32 %0, %0, %1\n")
                          : "+v"(a) : "v"(b) : "vcc"));
    }
    // 18: 20 x (v_cmp -> vcc, s_cbranch_vccnz not taken, v_add, v_add)
    {
        TIME(asm volatile(REP10("v_cmp_gt_u32 vcc, %1, %1\n s_cbranch_vccnz 1f\n v_add_u32 %0, %0, %1\n1:\n v_add_u32 %0, %0, %1\n"
                                "v_cmp_gt_u32 vcc, %1, %1\n s_cbranch_vccnz 2f\n v_add_u32 %0, %0, %1\n2:\n v_add_u32 %0, %0, %1\n")
                          : "+v"(a) : "v"(b) : "vcc"));
    }
    // 19: 100 dependent v_cndmask_b32 e32 (vcc), vcc rewritten by an independent v_cmp every 2
    TIME(asm volatile(REP10("v_cmp_gt_u32 vcc, %2, 7\n v_cndmask_b32 %0, %1, %0, vcc\n v_cndmask_b32 %0, %1, %0, vcc\n v_cmp_gt_u32 vcc, %2, 7\n v_cndmask_b32 %0, %1, %0, vcc\n v_cndmask_b32 %0, %1, %0, vcc\n"
                            "v_cmp_gt_u32 vcc, %2, 7\n v_cndmask_b32 %0, %1, %0, vcc\n v_cndmask_b32 %0, %1, %0, vcc\n v_cndmask_b32 %0, %1, %0, vcc\n")
                      : "+v"(a) : "v"(c), "v"(d) : "vcc"));
    // 20: 20 x dependent (v_cmp_e64 -> s_and_b64 -> v_cndmask_e64)
    TIME(asm volatile(REP10("v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n v_cndmask_b32_e64 %0, %1, %0, s[42:43]\n"
                            "v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n v_cndmask_b32_e64 %0, %1, %0, s[42:43]\n")
                      : "+v"(a) : "v"(c), "v"(d) : "s40", "s41", "s42", "s43", "scc"));
    // 21: 20 x dependent (v_cmp_e64 -> s_and_b64, 4 independent v_add, -> v_cndmask_e64)
    TIME(asm volatile(REP10("v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_cndmask_b32_e64 %0, %1, %0, s[42:43]\n"
                            "v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_add_u32 %3, %3, %2\n v_cndmask_b32_e64 %0, %1, %0, s[42:43]\n")
                      : "+v"(a), "+v"(e) : "v"(c), "v"(d) : "s40", "s41", "s42", "s43", "scc"));
    // 22: 20 x dependent (v_cmp_e64 -> v_cndmask_e64), for comparison with 20
    TIME(asm volatile(REP10("v_cmp_lt_u32_e64 s[40:41], %0, %2\n v_cndmask_b32_e64 %0, %1, %0, s[40:41]\n"
                            "v_cmp_lt_u32_e64 s[40:41], %0, %2\n v_cndmask_b32_e64 %0, %1, %0, s[40:41]\n")
                      : "+v"(a) : "v"(c), "v"(d) : "s40", "s41"));
    // 23: 20 x (v_cmp_e64 -> s_and_b64 -> s_cbranch_scc taken)
    TIME(asm volatile(REP10("v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n s_cbranch_scc1 1f\n v_add_u32 %0, %0, %1\n1:\n"
                            "v_cmp_lt_u32_e64 s[40:41], %0, %2\n s_and_b64 s[42:43], s[40:41], exec\n s_cbranch_scc1 2f\n v_add_u32 %0, %0, %1\n2:\n")
                      : "+v"(a) : "v"(c), "v"(d) : "s40", "s41", "s42", "s43", "scc"));
    if (a == 0x12345 && lane == 77) out[0] = a + (uint32_t)w;
}

int main() {
    unsigned long long* d;
    const int nblk = 1024;   // 4 per CU: one wave per SIMD
    hipMalloc(&d, nblk * 32 * 8);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, 3u);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, 3u);
    hipDeviceSynchronize();
    static unsigned long long h[nblk * 32];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* names[] = {"100 dep v_add", "100 v_add 4 chains", "100 dep v_lshrrev_b64", "100 dep v_cndmask vcc",
                           "100 x (v_cmp sgpr + dep cndmask)", "20 dep ds_read_b32", "20 x (ds_or + ds_read)", "100 dep s_add",
                           "50 v_add + 50 s_add", "6 ds_read2st64 + wait", "20 ds_or + wait", "20 ds_write + wait",
                           "10 x (4 ds_or + dep ds_read)", "10 x (4 ds_write + dep ds_read)", "100 dep cndmask_e64 fixed sgpr",
                           "20 x (scmp + taken cbranch + 2 vadd)", "20 x (scmp + not-taken cbranch + 2 vadd)",
                           "20 x (vcmp + taken vccz + 1 vadd)", "20 x (vcmp + not-taken vccnz + 2 vadd)",
                           "30 vcmp + 70 dep cndmask vcc", "20 x (vcmp -> s_and -> cndmask)",
                           "20 x (vcmp -> s_and, 4 vadd, cndmask)", "20 x (vcmp -> cndmask)", "20 x (vcmp -> s_and -> cbranch)"};
    for (int i = 0; i < 24; ++i) {
        double s = 0; unsigned long long mn = ~0ull;
        for (int b = 0; b < nblk; ++b) { s += h[b * 32 + i]; mn = h[b * 32 + i] < mn ? h[b * 32 + i] : mn; }
        printf("%-36s avg %8.1f  min %6llu cycles\n", names[i], s / nblk, mn);
    }
    return 0;
}
