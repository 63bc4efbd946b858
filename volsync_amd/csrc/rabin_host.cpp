// rabin_host.cpp -- GF(2)[x] arithmetic for the chunker tables (host side).
// Restates github.com/restic/chunker@v0.4.0 polynomials.go (Pol.Deg, Pol.Mod,
// Pol.Irreducible) and chunker.go fillTables/appendByte.
#include "internal.hpp"

namespace vsgpu {

int pol_deg(uint64_t p) { return p ? 63 - __builtin_clzll(p) : -1; }

uint64_t pol_mod(uint64_t x, uint64_t d) {
    if (!x) return 0;
    const int dd = pol_deg(d);
    while (x && pol_deg(x) >= dd) x ^= d << (pol_deg(x) - dd);
    return x;
}

static uint64_t append_byte(uint64_t h, uint8_t b, uint64_t pol) {
    return pol_mod((h << 8) | b, pol);
}

// 128-bit carry-less product reduced mod p (p of degree <= 63)
static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t p) {
    const int dp = pol_deg(p);
    uint64_t r = 0;
    a = pol_mod(a, p);
    for (int i = 63; i >= 0; --i) {
        r <<= 1;  // r = r * x mod p (r < 2^dp before the shift)
        if ((r >> dp) & 1) r ^= p;
        if ((b >> i) & 1) r ^= a;
    }
    return r;
}

static uint64_t gcd(uint64_t a, uint64_t b) {
    while (b) {
        uint64_t t = pol_mod(a, b);
        a = b;
        b = t;
    }
    return a;
}

// Ben-Or: irreducible iff gcd(x^(2^i) - x mod p, p) == 1 for i = 1..deg/2
bool pol_irreducible(uint64_t p) {
    const int d = pol_deg(p);
    if (d < 1) return false;
    uint64_t xp = 2;  // x
    for (int i = 1; i <= d / 2; ++i) {
        xp = mulmod(xp, xp, p);
        if (gcd(p, xp ^ 2) != 1) return false;
    }
    return true;
}

void pol_tables(uint64_t pol, uint64_t out_tab[256], uint64_t mod_tab[256]) {
    const int k = pol_deg(pol);
    for (int b = 0; b < 256; ++b) {
        uint64_t h = append_byte(0, (uint8_t)b, pol);
        for (int i = 0; i < 63; ++i) h = append_byte(h, 0, pol);
        out_tab[b] = h;
    }
    for (int b = 0; b < 256; ++b)
        mod_tab[b] = pol_mod((uint64_t)b << k, pol) | ((uint64_t)b << k);
}

void pol_out8(uint64_t pol, const uint64_t out_tab[256], uint64_t out8[256]) {
    for (int b = 0; b < 256; ++b) out8[b] = append_byte(out_tab[b], 0, pol);
}

}  // namespace vsgpu
