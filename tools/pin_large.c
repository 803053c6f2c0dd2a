/*
 * pin_large.c -- CONTAINER-ONLY CHECKER (test infrastructure, never the product).
 *
 * Computes exact full-range answers of the reference scan for the two large
 * BASELINE configs, independently of the GPU library, so the GPU tests and
 * bench.py can assert equality instead of size-independent properties:
 *   configs[2]: msg = "cmu440-p1-" x 12 (120 B), [0, 2^34)
 *   configs[3]: msg = "bradfitz",                [0, 2^38)
 *
 * What it restates (paths relative to /root/reference, SRC = src/github.com/cmu440):
 *   bitcoin.Hash  SRC/bitcoin/hash.go:13-17   SHA-256("msg nonce"), BigEndian.Uint64(sum[0:8])
 *   miner scan    SRC/bitcoin/miner/miner.go:56-63   inclusive [lower, upper], strict '<'
 *                 (lowest nonce wins ties), identity (MaxUint64, 0)
 * SHA-256 (Go stdlib crypto/sha256, FIPS 180-4) runs on the x86 SHA extensions
 * (gcc -msha): the host compresses the constant "msg " prefix blocks once
 * (midstate), each nonce's tail is formed by an ASCII decimal counter, and a
 * two-block tail reuses its first block while that block's bytes are unchanged.
 * The range is cut into chunks handed to threads from a shared counter; each
 * chunk reports its own (hash, nonce) (scanned in ascending order, strict '<')
 * and the answer is the lexicographic min over chunks -- identical to the
 * serial first minimum.  Chunk results are appended to a checkpoint file, so
 * an interrupted run resumes where it stopped.
 *
 * It is checked against oracle/p1_oracle.c and Python hashlib before its
 * answers are trusted (tests/test_pin_large.py; tools/pin_large.py runs it).
 *
 * usage: pin_large <msg_hex> <lower> <upper> [threads] [chunk_log2] [checkpoint]
 * prints one JSON line {"hash":H,"nonce":N,"nonces":C,"seconds":S,"threads":T}.
 */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static const uint32_t IV256[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                  0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

/* SHA-NI state: s0 = (A,B,E,F), s1 = (C,D,G,H), lane 3 first */
typedef struct { __m128i s0, s1; } nistate;

static __m128i KV[16];

static nistate ni_from_words(const uint32_t h[8]) {
    nistate s;
    s.s0 = _mm_set_epi32((int)h[0], (int)h[1], (int)h[4], (int)h[5]);
    s.s1 = _mm_set_epi32((int)h[2], (int)h[3], (int)h[6], (int)h[7]);
    return s;
}

/* message words in lane order (lane 0 = W[4j]) from a 64-byte block */
static inline void ni_load(const uint8_t *blk, __m128i m[4]) {
    const __m128i bswap = _mm_set_epi8(12, 13, 14, 15, 8, 9, 10, 11, 4, 5, 6, 7, 0, 1, 2, 3);
    for (int j = 0; j < 4; ++j) m[j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk + 16 * j)), bswap);
}

/* one FIPS 180-4 compression of the block held in m[0..3] into st */
static inline __attribute__((always_inline)) nistate ni_compress(nistate st, const __m128i min[4]) {
    __m128i m[4] = {min[0], min[1], min[2], min[3]};
    __m128i s0 = st.s0, s1 = st.s1;
#pragma GCC unroll 16
    for (int i = 0; i < 16; ++i) {
        __m128i msg = _mm_add_epi32(m[i & 3], KV[i]);
        s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
        if (i >= 3 && i <= 14) { /* W[4(i+1) .. 4(i+1)+3] */
            __m128i t = _mm_alignr_epi8(m[i & 3], m[(i - 1) & 3], 4);
            m[(i + 1) & 3] = _mm_add_epi32(m[(i + 1) & 3], t);
            m[(i + 1) & 3] = _mm_sha256msg2_epu32(m[(i + 1) & 3], m[i & 3]);
        }
        msg = _mm_shuffle_epi32(msg, 0x0E);
        s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
        if (i >= 1 && i <= 12) m[(i - 1) & 3] = _mm_sha256msg1_epu32(m[(i - 1) & 3], m[i & 3]);
    }
    nistate r;
    r.s0 = _mm_add_epi32(s0, st.s0);
    r.s1 = _mm_add_epi32(s1, st.s1);
    return r;
}

/* BigEndian.Uint64(sum[0:8]) = H0<<32 | H1 = lanes 3,2 of s0 */
static inline uint64_t ni_top64(nistate s) { return (uint64_t)_mm_extract_epi64(s.s0, 1); }

/* scalar compression for the midstate (runs once) */
#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void compress_scalar(uint32_t s[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) | ((uint32_t)blk[4 * t + 2] << 8) |
               (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; ++t)
        w[t] = w[t - 16] + (ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3)) + w[t - 7] +
               (ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10));
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t t1 = h + (ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
        uint32_t t2 = (ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

/* ---------------- the scan ---------------- */
static uint8_t *g_msg;
static size_t g_len;
static uint32_t g_mid[8];    /* state after the floor((L+1)/64) constant blocks */
static size_t g_r;           /* (L+1) mod 64: constant bytes that start the tail */
static uint8_t g_rbytes[64]; /* those bytes (msg tail + ' ') */

static unsigned ndigits(uint64_t v) {
    unsigned d = 1;
    while (v >= 10u) { v /= 10u; ++d; }
    return d;
}

static uint64_t pow10u(unsigned k) {
    uint64_t p = 1;
    while (k--) p *= 10u;
    return p;
}

typedef struct { uint64_t h, n; } pkey_t;
static inline int key_lt(pkey_t a, pkey_t b) { return a.h < b.h || (a.h == b.h && a.n < b.n); }
static inline pkey_t key_min(pkey_t a, pkey_t b) { return key_lt(b, a) ? b : a; }
static int g_vec = 1; /* PIN_NO_AVX512=1: SHA-NI only (cross-check of the two paths) */

/* Scan [lo, hi] (all nonces with the same digit count d), ascending, strict '<'. */
static pkey_t scan_decade(uint64_t lo, uint64_t hi, unsigned d, pkey_t best) {
    uint8_t tail[128];
    const size_t q = g_r + d;                    /* bytes before 0x80 */
    const size_t tl = (q + 9 <= 64) ? 64 : 128;  /* B_tail = 1 or 2 */
    memset(tail, 0, sizeof tail);
    memcpy(tail, g_rbytes, g_r);
    tail[q] = 0x80;
    const uint64_t bits = (uint64_t)(g_len + 1 + d) * 8u;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    /* digits of lo */
    uint8_t *dig = tail + g_r;
    {
        uint64_t v = lo;
        for (int i = (int)d - 1; i >= 0; --i) { dig[i] = (uint8_t)('0' + v % 10u); v /= 10u; }
    }
    const size_t upos = q - 1;                  /* units digit byte */
    const int ublk = (int)(upos / 64);          /* block of the units digit */
    const int uw = (int)((upos % 64) / 4);      /* its word */
    const int ush = (int)(3 - (upos % 4)) * 8;  /* its bit shift inside the word */
    const nistate mid = ni_from_words(g_mid);
    const int two = tl == 128;
    uint8_t blk0_prev[64];
    int have_prev = 0;
    nistate after0 = mid;
    __m128i delta[10]; /* the units digit u XORed into its word ('0' ^ u = '0' + u) */
    for (unsigned u = 0; u < 10; ++u) {
        uint32_t lanes[4] = {0, 0, 0, 0};
        lanes[uw & 3] = u << ush;
        delta[u] = _mm_loadu_si128((const __m128i *)lanes);
    }
    uint64_t n = lo;
    for (;;) {
        /* a group: every nonce from n to the next multiple of 10 (or hi) */
        const unsigned u0 = (unsigned)(n % 10u);
        uint64_t cnt = 10u - u0;
        if (hi - n < cnt - 1) cnt = hi - n + 1;
        dig[d - 1] = '0';
        __m128i m0[4], m1[4];
        if (two && ublk == 1) {
            if (!have_prev || memcmp(blk0_prev, tail, 64) != 0) {
                __m128i b0[4];
                ni_load(tail, b0);
                after0 = ni_compress(mid, b0);
                memcpy(blk0_prev, tail, 64);
                have_prev = 1;
            }
            ni_load(tail + 64, m1);
            for (unsigned u = u0; u < u0 + cnt; ++u) {
                __m128i mm[4] = {m1[0], m1[1], m1[2], m1[3]};
                mm[uw >> 2] = _mm_xor_si128(mm[uw >> 2], delta[u]);
                const uint64_t h = ni_top64(ni_compress(after0, mm));
                if (h < best.h) { best.h = h; best.n = n + (u - u0); }
            }
        } else {
            ni_load(tail, m0);
            if (two) ni_load(tail + 64, m1);
            for (unsigned u = u0; u < u0 + cnt; ++u) {
                __m128i mm[4] = {m0[0], m0[1], m0[2], m0[3]};
                mm[uw >> 2] = _mm_xor_si128(mm[uw >> 2], delta[u]);
                nistate s = ni_compress(mid, mm);
                if (two) s = ni_compress(s, m1);
                const uint64_t h = ni_top64(s);
                if (h < best.h) { best.h = h; best.n = n + (u - u0); }
            }
        }
        if (hi - n < cnt) break; /* n + cnt - 1 == hi */
        n += cnt;
        /* advance the decimal counter by one ten (carry into the higher digits) */
        int i = (int)d - 2;
        while (i >= 0 && dig[i] == '9') { dig[i] = '0'; --i; }
        if (i < 0) break; /* cannot happen inside one decade */
        dig[i]++;
    }
    return best;
}


/* ---------------- 16-lane AVX-512 path for 1-block tails ----------------
 * Lane j owns hi value h0 + j (the nonce's digits above the last kLoDigits)
 * and all lanes step the same lo in [0, 10^kLoDigits): nonce = hi*10^6 + lo.
 * Bytes of hi digits are per-lane constants; the lo digits are XORed in per
 * step as a broadcast (every lane has the same lo).  Same FIPS 180-4
 * arithmetic as compress_scalar, 16 blocks at a time. */
enum { kLoDigits = 6 };
static const uint64_t kLoSpan = 1000000u;

#define V16 __m512i
#define VROR(x, n) _mm512_ror_epi32((x), (n))
#define VX3(a, b, c) _mm512_ternarylogic_epi32((a), (b), (c), 0x96)

/* H0<<32|H1 of 16 lanes: out_lo = lanes 0..7, out_hi = lanes 8..15 */
static inline __attribute__((always_inline)) void v_compress_top(const V16 mid[8], const V16 win[16], __m512i *top_lo,
                                                                 __m512i *top_hi) {
    V16 w[16];
    for (int t = 0; t < 16; ++t) w[t] = win[t];
    V16 a = mid[0], b = mid[1], c = mid[2], d = mid[3], e = mid[4], f = mid[5], g = mid[6], h = mid[7];
#pragma GCC unroll 64
    for (int t = 0; t < 64; ++t) {
        V16 wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const V16 x15 = w[(t - 15) & 15], x2 = w[(t - 2) & 15];
            const V16 s0 = VX3(VROR(x15, 7), VROR(x15, 18), _mm512_srli_epi32(x15, 3));
            const V16 s1 = VX3(VROR(x2, 17), VROR(x2, 19), _mm512_srli_epi32(x2, 10));
            wt = _mm512_add_epi32(_mm512_add_epi32(w[t & 15], s0), _mm512_add_epi32(w[(t - 7) & 15], s1));
            w[t & 15] = wt;
        }
        const V16 S1 = VX3(VROR(e, 6), VROR(e, 11), VROR(e, 25));
        const V16 ch = _mm512_ternarylogic_epi32(e, f, g, 0xCA);
        const V16 t1 = _mm512_add_epi32(_mm512_add_epi32(h, S1),
                                        _mm512_add_epi32(ch, _mm512_add_epi32(_mm512_set1_epi32((int)K256[t]), wt)));
        const V16 S0 = VX3(VROR(a, 2), VROR(a, 13), VROR(a, 22));
        const V16 mj = _mm512_ternarylogic_epi32(a, b, c, 0xE8);
        h = g; g = f; f = e; e = _mm512_add_epi32(d, t1);
        d = c; c = b; b = a; a = _mm512_add_epi32(t1, _mm512_add_epi32(S0, mj));
    }
    const V16 H0 = _mm512_add_epi32(a, mid[0]), H1 = _mm512_add_epi32(b, mid[1]);
    /* interleave to u64 (H0 high, H1 low) */
    const __m512i lo = _mm512_unpacklo_epi32(H1, H0); /* lanes 0,1,4,5,8,9,12,13 */
    const __m512i hi = _mm512_unpackhi_epi32(H1, H0); /* lanes 2,3,6,7,10,11,14,15 */
    *top_lo = lo;
    *top_hi = hi;
}

/* lane order of the two u64 vectors above */
static const int kLaneOfLo[8] = {0, 1, 4, 5, 8, 9, 12, 13};
static const int kLaneOfHi[8] = {2, 3, 6, 7, 10, 11, 14, 15};

/* 16 hi values h0..h0+15 (all of d digits in total, d >= kLoDigits+1, 1-block tail), every lo. */
static pkey_t scan_vec16(uint64_t h0, unsigned d, pkey_t best) {
    const size_t q = g_r + d;
    uint32_t base[16][16]; /* [lane][word] */
    for (int j = 0; j < 16; ++j) {
        uint8_t tail[64];
        memset(tail, 0, sizeof tail);
        memcpy(tail, g_rbytes, g_r);
        uint64_t v = (h0 + (uint64_t)j) * kLoSpan; /* lo digits '0' */
        for (int i = (int)d - 1; i >= 0; --i) { tail[g_r + (size_t)i] = (uint8_t)('0' + v % 10u); v /= 10u; }
        tail[q] = 0x80;
        const uint64_t bits = (uint64_t)(g_len + 1 + d) * 8u;
        for (int i = 0; i < 8; ++i) tail[63 - i] = (uint8_t)(bits >> (8 * i));
        for (int w = 0; w < 16; ++w)
            base[j][w] = ((uint32_t)tail[4 * w] << 24) | ((uint32_t)tail[4 * w + 1] << 16) |
                         ((uint32_t)tail[4 * w + 2] << 8) | (uint32_t)tail[4 * w + 3];
    }
    V16 bw[16], mid[8];
    for (int w = 0; w < 16; ++w) {
        uint32_t col[16];
        for (int j = 0; j < 16; ++j) col[j] = base[j][w];
        bw[w] = _mm512_loadu_si512((const void *)col);
    }
    for (int i = 0; i < 8; ++i) mid[i] = _mm512_set1_epi32((int)g_mid[i]);
    /* lo digit i (0 = most significant of the 6) sits at byte g_r + d - 6 + i */
    int lw[kLoDigits], lsh[kLoDigits];
    for (int i = 0; i < kLoDigits; ++i) {
        const size_t pos = g_r + d - kLoDigits + (size_t)i;
        lw[i] = (int)(pos / 4);
        lsh[i] = (int)(3 - pos % 4) * 8;
    }
    const int wfirst = lw[0], wlast = lw[kLoDigits - 1];
    __m512i bh_lo = _mm512_set1_epi64(-1), bh_hi = _mm512_set1_epi64(-1);
    __m512i bl_lo = _mm512_setzero_si512(), bl_hi = _mm512_setzero_si512(); /* best lo per lane */
    unsigned digs[kLoDigits] = {0, 0, 0, 0, 0, 0};
    for (uint64_t lo = 0; lo < kLoSpan; ++lo) {
        uint32_t x[16] = {0};
        for (int i = 0; i < kLoDigits; ++i) x[lw[i]] ^= digs[i] << lsh[i];
        V16 win[16];
        for (int w = 0; w < 16; ++w) win[w] = bw[w];
        for (int w = wfirst; w <= wlast; ++w) win[w] = _mm512_xor_si512(bw[w], _mm512_set1_epi32((int)x[w]));
        __m512i tl, th;
        v_compress_top(mid, win, &tl, &th);
        /* strict '<' per lane, ascending lo: the first minimum of each lane */
        const __mmask8 ml = _mm512_cmplt_epu64_mask(tl, bh_lo), mh = _mm512_cmplt_epu64_mask(th, bh_hi);
        if (ml | mh) {
            const __m512i lov = _mm512_set1_epi64((long long)lo);
            bh_lo = _mm512_mask_mov_epi64(bh_lo, ml, tl);
            bl_lo = _mm512_mask_mov_epi64(bl_lo, ml, lov);
            bh_hi = _mm512_mask_mov_epi64(bh_hi, mh, th);
            bl_hi = _mm512_mask_mov_epi64(bl_hi, mh, lov);
        }
        /* decimal increment of the lo digits */
        int i = kLoDigits - 1;
        while (i >= 0 && digs[i] == 9) { digs[i] = 0; --i; }
        if (i >= 0) digs[i]++;
    }
    uint64_t hl[8], hh[8], ll[8], lh[8];
    _mm512_storeu_si512((void *)hl, bh_lo);
    _mm512_storeu_si512((void *)hh, bh_hi);
    _mm512_storeu_si512((void *)ll, bl_lo);
    _mm512_storeu_si512((void *)lh, bl_hi);
    for (int k = 0; k < 8; ++k) {
        const pkey_t a = {hl[k], (h0 + (uint64_t)kLaneOfLo[k]) * kLoSpan + ll[k]};
        const pkey_t b = {hh[k], (h0 + (uint64_t)kLaneOfHi[k]) * kLoSpan + lh[k]};
        if (key_lt(a, best)) best = a;
        if (key_lt(b, best)) best = b;
    }
    return best;
}

/* [lo, hi] inclusive, any digit counts: cut at powers of ten */
static pkey_t scan_range(uint64_t lo, uint64_t hi) {
    pkey_t best = {UINT64_MAX, UINT64_MAX};
    uint64_t a = lo;
    for (;;) {
        const unsigned d = ndigits(a);
        const uint64_t top = d >= 20 ? UINT64_MAX : pow10u(d) - 1;
        const uint64_t b = hi < top ? hi : top;
        if (g_vec && d > kLoDigits && g_r + d + 9 <= 64) {
            /* whole 10^6 blocks in groups of 16 on AVX-512, the rest on SHA-NI */
            const uint64_t h_first = a / kLoSpan + (a % kLoSpan ? 1 : 0);
            const uint64_t h_end = b / kLoSpan + (b % kLoSpan == kLoSpan - 1 ? 1 : 0); /* exclusive */
            uint64_t h = h_first;
            if (h_end > h_first && h_end - h_first >= 16) {
                if (a < h_first * kLoSpan) best = key_min(best, scan_decade(a, h_first * kLoSpan - 1, d, best));
                for (; h_end - h >= 16; h += 16) best = scan_vec16(h, d, best);
                if (h * kLoSpan <= b) best = key_min(best, scan_decade(h * kLoSpan, b, d, best));
            } else {
                best = scan_decade(a, b, d, best);
            }
        } else {
            best = scan_decade(a, b, d, best);
        }
        if (b == hi) break;
        a = b + 1;
    }
    return best;
}

/* ---------------- threads, chunks, checkpoint ---------------- */
static uint64_t g_lo, g_hi, g_chunk;
static uint64_t g_nchunks;
static atomic_ullong g_next;
static pkey_t *g_res;
static unsigned char *g_done;
static FILE *g_ckpt;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_finished;
static double g_t0;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void chunk_bounds(uint64_t c, uint64_t *a, uint64_t *b) {
    *a = g_lo + c * g_chunk;
    *b = (g_hi - *a < g_chunk - 1) ? g_hi : *a + g_chunk - 1;
}

static void *worker(void *arg) {
    (void)arg;
    for (;;) {
        const uint64_t c = atomic_fetch_add(&g_next, 1);
        if (c >= g_nchunks) break;
        if (g_done[c]) continue;
        uint64_t a, b;
        chunk_bounds(c, &a, &b);
        const pkey_t k = scan_range(a, b);
        pthread_mutex_lock(&g_mu);
        g_res[c] = k;
        g_done[c] = 1;
        ++g_finished;
        if (g_ckpt) {
            fprintf(g_ckpt, "%llu %llu %llu %llu\n", (unsigned long long)a, (unsigned long long)b,
                    (unsigned long long)k.h, (unsigned long long)k.n);
            fflush(g_ckpt);
        }
        if (g_nchunks >= 64 && g_finished % (g_nchunks / 64) == 0)
            fprintf(stderr, "pin_large: %llu/%llu chunks, %.1f s\n", (unsigned long long)g_finished,
                    (unsigned long long)g_nchunks, now_s() - g_t0);
        pthread_mutex_unlock(&g_mu);
    }
    return NULL;
}

static int unhex(const char *s, uint8_t **out, size_t *len) {
    size_t n = strlen(s);
    if (n % 2) return -1;
    *len = n / 2;
    *out = (uint8_t *)malloc(*len + 1);
    for (size_t i = 0; i < *len; ++i) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
        (*out)[i] = (uint8_t)v;
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <msg_hex> <lower> <upper> [threads] [chunk_log2] [checkpoint]\n", argv[0]);
        return 2;
    }
    if (unhex(argv[1], &g_msg, &g_len) != 0) { fprintf(stderr, "bad hex\n"); return 2; }
    g_lo = strtoull(argv[2], NULL, 10);
    g_hi = strtoull(argv[3], NULL, 10);
    int nth = argc > 4 ? atoi(argv[4]) : 8;
    {
        const char *nv = getenv("PIN_NO_AVX512");
        g_vec = !(nv && nv[0] == '1');
    }
    const int clog = argc > 5 ? atoi(argv[5]) : 26;
    const char *ck = argc > 6 ? argv[6] : NULL;
    for (int i = 0; i < 16; ++i)
        KV[i] = _mm_set_epi32((int)K256[4 * i + 3], (int)K256[4 * i + 2], (int)K256[4 * i + 1], (int)K256[4 * i]);
    /* midstate over the constant prefix blocks of msg ' ' */
    memcpy(g_mid, IV256, sizeof g_mid);
    const size_t pre = g_len + 1;
    uint8_t *buf = (uint8_t *)malloc(pre);
    memcpy(buf, g_msg, g_len);
    buf[g_len] = ' ';
    size_t off = 0;
    for (; off + 64 <= pre; off += 64) compress_scalar(g_mid, buf + off);
    g_r = pre - off;
    memcpy(g_rbytes, buf + off, g_r);
    free(buf);
    if (g_lo > g_hi) {
        printf("{\"hash\": %llu, \"nonce\": 0, \"nonces\": 0, \"seconds\": 0, \"threads\": 0}\n",
               (unsigned long long)UINT64_MAX);
        return 0;
    }
    g_chunk = 1ull << clog;
    g_nchunks = (g_hi - g_lo) / g_chunk + 1;
    g_res = (pkey_t *)calloc(g_nchunks, sizeof(pkey_t));
    g_done = (unsigned char *)calloc(g_nchunks, 1);
    if (ck) {
        FILE *f = fopen(ck, "r");
        if (f) { /* resume: reuse chunks whose bounds match this run's chunking */
            unsigned long long a, b, h, n;
            while (fscanf(f, "%llu %llu %llu %llu", &a, &b, &h, &n) == 4) {
                if (a < g_lo || ((uint64_t)a - g_lo) % g_chunk) continue;
                const uint64_t c = ((uint64_t)a - g_lo) / g_chunk;
                uint64_t ea, eb;
                if (c >= g_nchunks) continue;
                chunk_bounds(c, &ea, &eb);
                if (ea != a || eb != b) continue;
                g_res[c].h = h; g_res[c].n = n; g_done[c] = 1;
                ++g_finished;
            }
            fclose(f);
        }
        g_ckpt = fopen(ck, "a");
    }
    if (nth < 1) nth = 1;
    g_t0 = now_s();
    pthread_t *tid = (pthread_t *)calloc((size_t)nth, sizeof(pthread_t));
    for (int t = 0; t < nth; ++t) pthread_create(&tid[t], NULL, worker, NULL);
    for (int t = 0; t < nth; ++t) pthread_join(tid[t], NULL);
    const double secs = now_s() - g_t0;
    pkey_t best = {UINT64_MAX, UINT64_MAX};
    for (uint64_t c = 0; c < g_nchunks; ++c)
        if (key_lt(g_res[c], best)) best = g_res[c];
    if (best.h == UINT64_MAX) best.n = 0; /* identity (MaxUint64, 0) of miner.go:56 */
    printf("{\"hash\": %llu, \"nonce\": %llu, \"nonces\": %llu, \"seconds\": %.3f, \"threads\": %d}\n",
           (unsigned long long)best.h, (unsigned long long)best.n, (unsigned long long)(g_hi - g_lo + 1), secs, nth);
    if (g_ckpt) fclose(g_ckpt);
    return 0;
}
