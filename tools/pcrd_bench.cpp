// Host-only timing harness for T2Enc::allocate (PCRD rate control) on the C3 geometry
// (8192x8192, 3 components, 12-bit, 9/7, 3 layers -r 40,20,10) with synthetic pass
// records.  No GPU call is made.  Build: tools/pcrd_bench.sh
#ifndef ENGINE_SRC
#define ENGINE_SRC "../grok_amd/csrc/gk_engine.cpp"
#endif
#include ENGINE_SRC
#include <random>

int main(int argc, char** argv) {
    Plan P;
    P.w = P.h = argc > 1 ? (uint32_t)atoi(argv[1]) : 8192;
    P.nc = 3; P.prec = 12; P.sgnd = 0;
    P.p.irrev = 1; P.p.nlayers = 3; P.p.rates[0] = 40; P.p.rates[1] = 20; P.p.rates[2] = 10;
    for (int i = 0; i < GK_MAXRLVLS; ++i) { P.p.prcw[i] = 15; P.p.prch[i] = 15; }
    build_plan(P);
    const uint32_t nb = (uint32_t)P.blocks.size();
    std::mt19937 rng(7);
    std::vector<uint32_t> info(4 * (size_t)nb);
    std::vector<GkPass> passes;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t bnb = P.blocks[b].band_numbps;
        const uint32_t nbps = bnb > 4 ? bnb - 4 + rng() % 5 : bnb;
        const uint32_t np = nbps ? 3 * nbps - 2 : 0;
        info[4 * b] = nbps; info[4 * b + 1] = np; info[4 * b + 3] = (uint32_t)passes.size();
        uint32_t r = 0; double d = 0, sd = 1e6 * (1 + rng() % 100);
        for (uint32_t q = 0; q < np; ++q) {
            const uint32_t dr = (q < 3 * nbps / 2) ? 1 + rng() % 8 : 40 + rng() % 200;
            r += dr; d += sd * dr; sd *= 0.55 + 0.1 * (rng() % 100) / 100.0;
            passes.push_back({r, dr, d});
        }
        info[4 * b + 2] = r;
    }
    if (argc > 2) {   // pass records dumped by the engine (GK_DUMP_PASSES) for this geometry
        FILE* f = fopen(argv[2], "rb");
        uint32_t hdr[2];
        if (!f || fread(hdr, 4, 2, f) != 2 || hdr[0] != nb) { fprintf(stderr, "bad dump\n"); return 1; }
        passes.resize(hdr[1]);
        if (fread(info.data(), 16, nb, f) != nb || fread(passes.data(), sizeof(GkPass), hdr[1], f) != hdr[1]) return 1;
        fclose(f);
    }
    printf("blocks %u passes %zu\n", nb, passes.size());
    {   // host pool dispatch: an empty job over the pool's threads, and a 49,152-item light job
        const size_t n = host_pool().size();
        std::atomic<uint64_t> sink{0};
        for (int rep = 0; rep < 4; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 1000; ++i) host_pool().run(n, [&](size_t q) { sink += q; });
            auto t1 = std::chrono::steady_clock::now();
            for (int i = 0; i < 100; ++i)
                host_pool().run(24, [&](size_t q) { uint64_t a = 0; for (size_t k = 0; k < 2048; ++k) a += k * q; sink += a; });
            auto t2 = std::chrono::steady_clock::now();
            printf("pool %zu threads: empty dispatch %.2f us, 24 x 2048 items %.2f us\n", n,
                   std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000,
                   std::chrono::duration<double, std::micro>(t2 - t1).count() / 100);
        }
    }
    for (int it = 0; it < 8; ++it) {
        T2Enc T2(P, info.data(), passes.data(), 0, 1);
        T2.serial = getenv("PCRD_SERIAL") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        T2.allocate(200);
        uint64_t h = 0;
        for (size_t i = 0; i < T2.lnp.size(); ++i) h = h * 1000003u + T2.lnp[i];
#ifdef PCRD_TRACE
        printf("scans %llu passes %llu\n", (unsigned long long)g_scans.load(), (unsigned long long)g_scan_passes.load());
#endif
        printf("allocate %.2f ms (layer pass counts hash %016llx)\n",
               std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), (unsigned long long)h);
    }
}
