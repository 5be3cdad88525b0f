// Host-only stress test of the engine's HostPool (gk_engine.cpp): many back-to-back dispatches
// of varying sizes, each item must run exactly once per dispatch.  Build: see tools/pcrd_bench.sh
// (same link line); run with no arguments.
#ifndef ENGINE_SRC
#define ENGINE_SRC "../grok_amd/csrc/gk_engine.cpp"
#endif
#include ENGINE_SRC
#include <random>

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200000;
    std::mt19937 rng(1);
    std::vector<std::atomic<uint32_t>> hits(5000);
    uint64_t bad = 0;
    for (int it = 0; it < iters; ++it) {
        const size_t n = 1 + rng() % (it % 7 == 0 ? 4999 : 40);
        const uint32_t spin = rng() % 64;
        for (size_t i = 0; i < n; ++i) hits[i].store(0, std::memory_order_relaxed);
        host_pool().run(n, [&](size_t i) {
            volatile uint32_t x = 0;
            for (uint32_t k = 0; k < spin * (i % 3); ++k) x = x + k;
            hits[i].fetch_add(1, std::memory_order_relaxed);
        });
        for (size_t i = 0; i < n; ++i) bad += hits[i].load() != 1;
        if (bad) { printf("iteration %d: %llu items not run exactly once\n", it, (unsigned long long)bad); return 1; }
    }
    // an error in a worker reaches the caller
    bool caught = false;
    try { host_pool().run(100, [&](size_t i) { if (i == 77) throw GkError("item 77"); }); } catch (const GkError& e) { caught = e.msg == "item 77"; }
    printf("%d dispatches ok, error propagated: %s\n", iters, caught ? "yes" : "NO");
    return caught ? 0 : 1;
}
