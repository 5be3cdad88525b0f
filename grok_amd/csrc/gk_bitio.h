// gk_bitio.h — packet-header bit reader for the T2 decoder (host).
//
// Packet headers are bit-stuffed (ISO 15444-1 B.10.1; Grok BitIO::read / bytein, BitIO.cpp:
// 35-52, 104-132): a byte that follows 0xFF carries only 7 bits.  The reader keeps up to 64
// unread bits MSB-aligned in one register, refilled a byte at a time, so a field of n bits is
// one shift and a run of equal bits (tag-tree zeros, comma code ones) is one count of leading
// zeros, instead of a loop per bit.  Bytes at or past `end` read as 0, like Grok's reader.
//
// align() (BitIO::inalign) gives the byte position after the header: the byte holding the last
// bit taken, plus the byte after it when that byte is 0xFF.  Bits loaded ahead are given back
// by walking the loaded bytes backwards (each byte's width follows from the byte before it).
//
// Src provides `const uint8_t* span(size_t i, size_t& lo, size_t& hi)`: a contiguous window
// [lo, hi) holding byte i (i < Src::len), as ByteSrc does for host, device-page or fetched-range
// streams.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <algorithm>
#include <vector>

template <class Src>
struct PktBitReader {
    Src& s;
    size_t off;          // next byte to load (after align(): the packet body)
    size_t end;          // the tile part's end: bytes past it read as 0
    size_t start;
    uint64_t acc = 0;    // unread bits, MSB first
    int nb = 0;          // valid bits in acc
    uint32_t prev = 0;   // the last byte loaded (0 before the first: the first byte has 8 bits)
    const uint8_t* wp = nullptr;
    size_t wlo = 0, whi = 0;   // the cached window of s

    PktBitReader(Src& src, size_t o, size_t e) : s(src), off(o), end(e), start(o) {}

    inline uint32_t value(size_t i) {   // byte i of the header stream (0 at or past end)
        if (i >= end || i >= s.len) return 0;
        if (i - wlo >= whi - wlo) wp = s.span(i, wlo, whi);
        return wp[i - wlo];
    }
    inline void refill() {   // to more than 56 valid bits
        while (nb <= 56) {
            const uint32_t b = value(off);
            ++off;
            const int w = prev == 0xff ? 7 : 8;
            acc |= (uint64_t)(b & ((1u << w) - 1)) << (64 - nb - w);
            nb += w;
            prev = b;
        }
    }
    inline uint32_t read(int n) {   // 0 <= n <= 32
        if (n <= 0) return 0;
        if (nb < n) refill();
        const uint32_t v = (uint32_t)(acc >> (64 - n));
        acc <<= n;
        nb -= n;
        return v;
    }
    // Up to `limit` bits equal to `bit`; when a different bit comes first it is consumed too and
    // `ended` is set (what a loop of read(1) until the other bit would read).
    inline uint32_t run(uint32_t bit, uint32_t limit, bool& ended) {
        uint32_t n = 0;
        ended = false;
        for (;;) {
            if (nb <= 56) refill();
            const uint64_t x = bit ? ~acc : acc;   // the run is x's leading zeros
            const uint32_t z = std::min<uint32_t>(x ? (uint32_t)__builtin_clzll(x) : 64u, (uint32_t)nb);
            if (n + z >= limit) {
                const uint32_t k = limit - n;   // k <= z <= nb < 64 here unless the run fills acc
                if (k >= 64) { acc = 0; nb = 0; } else { acc <<= k; nb -= (int)k; }
                return limit;
            }
            if (z < (uint32_t)nb) {   // the run ends inside the register: take it and the other bit
                n += z;
                acc = (acc << z) << 1;
                nb -= (int)z + 1;
                ended = true;
                return n;
            }
            n += z;   // every valid bit belongs to the run
            acc = 0;
            nb = 0;
        }
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
    uint32_t commacode() { bool e; return run(1, 0xffffffffu, e); }
    void align() {
        // give back the bytes loaded ahead, then step past the byte holding the last bit taken
        // (and past the stuffing byte behind an 0xFF)
        size_t j = off;   // bytes [start, j) are loaded
        while (j > start) {
            const int w = (j - 1 > start && value(j - 2) == 0xff) ? 7 : 8;
            if (nb < w) break;
            nb -= w;
            --j;
        }
        if (j == start) { off = start; }
        else off = value(j - 1) == 0xff ? j + 1 : j;
        acc = 0; nb = 0; prev = 0;
    }
};

// Packet-header bit writer (BitIO::write / putbit / flush, BitIO.cpp:60-103): bits gather in a
// 64-bit register and leave a byte at a time once the next byte has begun, a byte after 0xFF
// holding 7 bits (MSB 0).  flush() writes the partial last byte (zero padded) and, when that
// byte is 0xFF, a 0x00 after it.
struct PktBitWriter {
    std::vector<uint8_t>& o;
    uint64_t acc = 0;    // pending bits, right-aligned (only the low nacc are meaningful)
    uint32_t nacc = 0;
    uint32_t w = 8;      // width of the byte being filled: 8, or 7 after 0xFF
    explicit PktBitWriter(std::vector<uint8_t>& out) : o(out) {}
    inline void put(uint32_t v, uint32_t k) {   // the low k <= 32 bits of v (higher bits zero)
        acc = (acc << k) | v;
        nacc += k;
        while (nacc > w) {   // a byte leaves when a bit of the next one exists (as Grok's lazy bytein)
            const uint32_t b = (uint32_t)(acc >> (nacc - w)) & ((1u << w) - 1);
            nacc -= w;
            o.push_back((uint8_t)b);
            w = b == 0xff ? 7 : 8;
        }
    }
    inline void putbit(uint32_t b) { put(b, 1); }
    inline void write(uint32_t v, int n) {
        if (n > 32) { put(0, (uint32_t)n - 32); n = 32; }
        put(n == 32 ? v : (v & ((1u << n) - 1)), (uint32_t)n);
    }
    void flush() {
        const uint32_t b = nacc ? (uint32_t)(acc << (w - nacc)) & ((1u << w) - 1) : 0u;
        o.push_back((uint8_t)b);
        if (b == 0xff) o.push_back(0);
        acc = 0; nacc = 0; w = 8;
    }
    void commacode(uint32_t n) {
        for (; n >= 31; n -= 31) put(0x7fffffffu, 31);
        put(((1u << n) - 1) << 1, n + 1);
    }
    void numpasses(uint32_t n) {
        if (n == 1) put(0, 1);
        else if (n == 2) put(2, 2);
        else if (n <= 5) put(0xc | (n - 3), 4);
        else if (n <= 36) put(0x1e0 | (n - 6), 9);
        else put(0xff80 | (n - 37), 16);
    }
};

// Grok's bounded packet-header BitIO as T2Compress::compressPacketSimulate uses it
// (BitIO(nullptr, max_bytes, true); BitIO.cpp:24-52, 80-122), emulated bit by bit for the
// rate control's budget test: writeByte counts a byte and fails when the count reaches buf_len
// (never when buf_len is 0, the count starting above it), leaving the pending byte and ct as
// they were; putbit fails with it, and write() returns at the first failed bit, dropping the
// rest of its value.  compressHeader checks every write but those inside putnumpasses and
// putcommacode (BitIO.cpp:144-178 return nothing): a failure there is swallowed, the header
// goes on (the next writeByte counts the same byte again, count buf_len + 1, and succeeds) and
// the count it reports runs past the budget.  Same interface as PktBitWriter.
struct GrkSimWriter {
    uint64_t offset = 0, buf_len;
    uint32_t buf = 0;
    int ct = 8;
    bool failed = false;      // a checked write or the flush reached the budget: the packet fails
    bool swallowed = false;   // the budget was reached inside a number-of-passes / comma code
    explicit GrkSimWriter(uint64_t len) : buf_len(len) {}
    inline bool write_byte() {
        ++offset;
        if (offset == buf_len) return false;
        ct = buf == 0xff ? 7 : 8;
        buf = 0;
        return true;
    }
    inline bool bit(uint32_t b) {
        if (ct == 0 && !write_byte()) return false;
        --ct;
        buf |= b << ct;
        return true;
    }
    inline bool bits(uint32_t v, uint32_t k) {
        for (int i = (int)k - 1; i >= 0; --i)
            if (!bit((v >> i) & 1)) return false;
        return true;
    }
    // checked writes (a run of tag-tree bits is a run of one-bit writes: failing at its first
    // failed bit is the same)
    inline void put(uint32_t v, uint32_t k) { if (!failed && !bits(v, k)) failed = true; }
    inline void putbit(uint32_t b) { put(b, 1); }
    inline void write(uint32_t v, int n) {
        if (n > 32) { put(0, (uint32_t)n - 32); n = 32; }
        put(n == 32 ? v : (v & ((1u << n) - 1)), (uint32_t)n);
    }
    void flush() {
        if (failed) return;
        if (!write_byte() || (ct == 7 && !write_byte())) failed = true;
    }
    // unchecked: BitIO::putcommacode writes one bit per call, putnumpasses its code in one call
    void commacode(uint32_t n) {
        if (failed) return;
        for (uint32_t i = 0; i < n; ++i) if (!bit(1)) swallowed = true;
        if (!bit(0)) swallowed = true;
    }
    void numpasses(uint32_t n) {
        if (failed) return;
        bool ok;
        if (n == 1) ok = bits(0, 1);
        else if (n == 2) ok = bits(2, 2);
        else if (n <= 5) ok = bits(0xc | (n - 3), 4);
        else if (n <= 36) ok = bits(0x1e0 | (n - 6), 9);
        else ok = bits(0xff80 | (n - 37), 16);
        if (!ok) swallowed = true;
    }
};
