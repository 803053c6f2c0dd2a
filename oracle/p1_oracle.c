/*
 * p1_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference's one data-parallel hot path, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and by
 * nothing else.  The product (libp1hip.so) never links, loads or calls it.
 *
 * What it restates (paths relative to /root/reference, SRC = src/github.com/cmu440):
 *   - bitcoin.Hash                SRC/bitcoin/hash.go:13-17
 *       bytes = fmt.Sprintf("%s %d", msg, nonce)      (hash.go:15)
 *       d     = sha256(bytes)                          (hash.go:14-16, Go stdlib)
 *       ret   = binary.BigEndian.Uint64(d[0:8])        (hash.go:16)
 *   - the miner scan              SRC/bitcoin/miner/miner.go:56-63
 *       min, minIndex := MaxUint64, 0                  (miner.go:56)
 *       for i := Lower; i <= Upper; i++ { if h < min { min, minIndex = h, i } }
 *     Documented divergence: Upper == 2^64-1 makes the Go loop wrap forever
 *     (i++ overflows); here the scan is inclusive and terminates.
 *
 * SHA-256 itself lives in Go's stdlib crypto/sha256 (Go 1.4.2 in the staff
 * binaries), which is NOT under /root/reference; this file restates FIPS 180-4.
 *
 * Parity pinning (see tests/test_oracle.py):
 *   - p1.pdf section 4.1 known answers: Hash("msg",0/1/2);
 *   - golden vectors the survey recorded from the compiled staff tester
 *     (bin/linux_amd64/mtest "Expecting result" lines);
 *   - independent hashlib fixtures in tests/golden/ (tests/golden/make_golden.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

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

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

/* FIPS 180-4 section 6.2.2: one compression of a 64-byte block into state s. */
static void compress(uint32_t s[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

/* Full SHA-256 (FIPS 180-4 section 5.1.1 padding) of buf[0..len). */
void p1o_sha256(const uint8_t *buf, size_t len, uint8_t out[32]) {
    uint32_t s[8];
    memcpy(s, IV256, sizeof s);
    size_t off = 0;
    for (; off + 64 <= len; off += 64) compress(s, buf + off);
    uint8_t tail[128];
    size_t rem = len - off;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, buf + off, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    compress(s, tail);
    if (tl == 128) compress(s, tail + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(s[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s[i] >> 8);
        out[4 * i + 3] = (uint8_t)s[i];
    }
}

/* Go's %d of a uint64: no sign, no padding, no leading zeros (hash.go:15). */
static size_t fmt_u64(uint64_t v, uint8_t *dst) {
    uint8_t tmp[20];
    size_t n = 0;
    do { tmp[n++] = (uint8_t)('0' + (v % 10u)); v /= 10u; } while (v);
    for (size_t i = 0; i < n; ++i) dst[i] = tmp[n - 1 - i];
    return n;
}

/* bitcoin.Hash(msg, nonce): hash.go:13-17.  `scratch` must hold len+21 bytes. */
static uint64_t hash_with(const uint8_t *msg, size_t len, uint64_t nonce, uint8_t *scratch) {
    if (len) memcpy(scratch, msg, len);
    scratch[len] = ' ';
    size_t n = len + 1 + fmt_u64(nonce, scratch + len + 1);
    uint8_t dg[32];
    p1o_sha256(scratch, n, dg);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | dg[i]; /* BigEndian.Uint64(Sum[0:8]) */
    return v;
}

uint64_t p1o_hash(const uint8_t *msg, size_t len, uint64_t nonce) {
    uint8_t small[256];
    uint8_t *scratch = (len + 21 <= sizeof small) ? small : (uint8_t *)malloc(len + 21);
    if (!scratch) return 0;
    uint64_t v = hash_with(msg, len, nonce, scratch);
    if (scratch != small) free(scratch);
    return v;
}

/* miner.go:56-63 over [lower, upper] inclusive; strict '<' keeps the lowest
 * nonce on ties; identity (MaxUint64, 0).  found = 1 if some hash < MaxUint64. */
static int scan_serial(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper,
                       uint64_t *out_hash, uint64_t *out_nonce) {
    uint64_t best = UINT64_MAX, bi = 0;
    int found = 0;
    if (lower <= upper) {
        uint8_t *scratch = (uint8_t *)malloc(len + 21);
        if (!scratch) return -1;
        for (uint64_t i = lower;; ++i) {
            uint64_t h = hash_with(msg, len, i, scratch);
            if (h < best) { best = h; bi = i; found = 1; }
            if (i == upper) break; /* inclusive, no wrap at 2^64-1 */
        }
        free(scratch);
    }
    *out_hash = best;
    *out_nonce = bi;
    return found;
}

int p1o_scan(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper,
             uint64_t *out_hash, uint64_t *out_nonce) {
    return scan_serial(msg, len, lower, upper, out_hash, out_nonce) < 0 ? -1 : 0;
}

typedef struct {
    const uint8_t *msg;
    size_t len;
    uint64_t lo, hi;
    uint64_t h, n;
    int found;
} job_t;

static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    j->found = scan_serial(j->msg, j->len, j->lo, j->hi, &j->h, &j->n);
    return NULL;
}

/* Same result as p1o_scan, split contiguously over `nthreads` host threads.
 * Contiguous shards + "first strict minimum across shards in order" keeps the
 * serial semantics exactly. */
int p1o_scan_mt(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper || nthreads <= 1) return p1o_scan(msg, len, lower, upper, out_hash, out_nonce);
    uint64_t span = upper - lower; /* count - 1, cannot overflow */
    if ((uint64_t)nthreads > span) nthreads = (int)span + 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *tid = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !tid) { free(jobs); free(tid); return -1; }
    uint64_t per = span / (uint64_t)nthreads, extra = span % (uint64_t)nthreads;
    uint64_t cur = lower;
    for (int t = 0; t < nthreads; ++t) {
        /* shard sizes sum to span+1 */
        uint64_t cnt = per + ((uint64_t)t < extra ? 1 : 0) + (t == nthreads - 1 ? 1 : 0);
        jobs[t].msg = msg; jobs[t].len = len; jobs[t].lo = cur; jobs[t].hi = cur + cnt - 1;
        cur += cnt;
        pthread_create(&tid[t], NULL, job_run, &jobs[t]);
    }
    uint64_t best = UINT64_MAX, bi = 0;
    int rc = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(tid[t], NULL);
        if (jobs[t].found < 0) rc = -1;
        else if (jobs[t].found && jobs[t].h < best) { best = jobs[t].h; bi = jobs[t].n; }
    }
    free(jobs);
    free(tid);
    *out_hash = best;
    *out_nonce = bi;
    return rc;
}
