// Randomised check of the T2 packet-header bit reader (grok_amd/csrc/gk_bitio.h) against
// a bit-at-a-time restatement of Grok's BitIO reader (BitIO.cpp: bytein / getbit / inalign: a
// byte after 0xFF carries 7 bits; bytes past the end read as 0).  Streams are dense in 0xFF
// bytes; the source hands out small windows so window changes are exercised.  Exit 0 = equal.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include "gk_bitio.h"

struct HostSrc {
    const uint8_t* p; size_t len; size_t win;
    const uint8_t* span(size_t i, size_t& lo, size_t& hi) {
        lo = i / win * win; hi = lo + win < len ? lo + win : len;
        return p + lo;
    }
};

struct RefReader {   // one bit at a time
    const std::vector<uint8_t>& b; size_t off, end; uint32_t buf = 0; int ct = 0;
    RefReader(const std::vector<uint8_t>& v, size_t o, size_t e) : b(v), off(o), end(e) {}
    void bytein() { ct = buf == 0xff ? 7 : 8; buf = off < end && off < b.size() ? b[off] : 0; ++off; }
    uint32_t bit() { if (ct == 0) bytein(); --ct; return (buf >> ct) & 1; }
    uint32_t read(int n) { uint32_t v = 0; for (int i = 0; i < n; ++i) v = (v << 1) | bit(); return v; }
    uint32_t run(uint32_t want, uint32_t limit, bool& ended) {
        uint32_t n = 0; ended = false;
        while (n < limit) { if (bit() != want) { ended = true; return n; } ++n; }
        return n;
    }
    uint32_t numpasses() {
        if (!read(1)) return 1;
        if (!read(1)) return 2;
        uint32_t n = read(2);
        if (n != 3) return n + 3;
        n = read(5);
        if (n != 31) return n + 6;
        return read(7) + 37;
    }
    void align() { if (buf == 0xff) bytein(); ct = 0; }
};

struct RefWriter {   // BitIO's writer, one bit at a time
    std::vector<uint8_t>& o; uint32_t buf = 0; int ct = 8;
    explicit RefWriter(std::vector<uint8_t>& v) : o(v) {}
    void wbyte() { o.push_back((uint8_t)buf); ct = buf == 0xff ? 7 : 8; buf = 0; }
    void putbit(uint32_t b) { if (ct == 0) wbyte(); --ct; buf |= b << ct; }
    void write(uint32_t v, int n) { for (int i = n - 1; i >= 0; --i) putbit((v >> i) & 1); }
    void flush() { wbyte(); if (ct == 7) wbyte(); }
    void commacode(uint32_t n) { for (uint32_t i = 0; i < n; ++i) putbit(1); putbit(0); }
    void numpasses(uint32_t n) {
        if (n == 1) write(0, 1);
        else if (n == 2) write(2, 2);
        else if (n <= 5) write(0xc | (n - 3), 4);
        else if (n <= 36) write(0x1e0 | (n - 6), 9);
        else write(0xff80 | (n - 37), 16);
    }
};

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)rs; }

int main() {
    long checks = 0;
    for (int it = 0; it < 20000; ++it) {
        const size_t n = 1 + rnd() % 200;
        std::vector<uint8_t> v(n);
        const uint32_t ffp = rnd() % 4;   // 0xFF density
        for (auto& x : v) {
            const uint32_t r = rnd() % 16;
            x = r < ffp * 3 ? 0xff : (r == 15 ? (uint8_t)(rnd() & 1 ? 0x00 : 0x8f + rnd() % 8) : (uint8_t)rnd());
        }
        const size_t o = rnd() % n, e = o + rnd() % (n - o + 8);   // end may lie past the data
        HostSrc src{v.data(), n, 1 + rnd() % 9};
        PktBitReader<HostSrc> a(src, o, e);
        RefReader r(v, o, e);
        const int ops = 1 + rnd() % 40;
        for (int k = 0; k < ops; ++k) {
            const uint32_t op = rnd() % 5;
            uint32_t x = 0, y = 0;
            if (op == 0) { const int m = rnd() % 33; x = a.read(m); y = r.read(m); }
            else if (op == 1) {
                const uint32_t bit = rnd() & 1, lim = 1 + (rnd() % 3 == 0 ? rnd() % 200 : rnd() % 12);
                bool ea, eb;
                x = a.run(bit, lim, ea); y = r.run(bit, lim, eb);
                if (ea != eb) { printf("run ended differs it=%d k=%d\n", it, k); return 1; }
            } else if (op == 2) { x = a.numpasses(); y = r.numpasses(); }
            else if (op == 3) { bool e1, e2; x = a.run(1, 0xffffffffu, e1); y = r.run(1, 0xffffffffu, e2); }
            else { a.align(); r.align(); x = (uint32_t)a.off; y = (uint32_t)r.off; break; }
            if (x != y) { printf("op %u differs it=%d k=%d: %u vs %u\n", op, it, k, x, y); return 1; }
            ++checks;
        }
        a.align(); r.align();
        if (a.off != r.off) { printf("align differs it=%d: %zu vs %zu\n", it, a.off, r.off); return 1; }
    }
    // writer: random field sequences (runs of ones make 0xFF bytes) through both writers
    for (int it = 0; it < 20000; ++it) {
        std::vector<uint8_t> a, b;
        PktBitWriter wa(a);
        RefWriter wb(b);
        const int ops = rnd() % 30;
        for (int k = 0; k < ops; ++k) {
            const uint32_t op = rnd() % 5;
            if (op == 0) { const int n = rnd() % 33; const uint32_t v = rnd() | (rnd() & 1 ? 0xff00ff00u : 0); wa.write(v, n); wb.write(v, n); }
            else if (op == 1) { const uint32_t n = rnd() % (rnd() % 4 == 0 ? 70 : 9); wa.commacode(n); wb.commacode(n); }
            else if (op == 2) { const uint32_t n = 1 + rnd() % 164; wa.numpasses(n); wb.numpasses(n); }
            else if (op == 3) { const uint32_t n = rnd() % 17; wa.put((1u << n) - 1, n); wb.write((1u << n) - 1, (int)n); }
            else { const uint32_t bit = rnd() & 1; wa.putbit(bit); wb.putbit(bit); }
        }
        wa.flush(); wb.flush();
        if (a != b) { printf("writer differs it=%d (%zu vs %zu bytes)\n", it, a.size(), b.size()); return 1; }
        ++checks;
    }
    printf("ok %ld checks\n", checks);
    return 0;
}
