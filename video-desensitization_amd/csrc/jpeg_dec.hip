// jpeg_dec.hip — baseline JPEG entropy decoding on the device (self-synchronising
// parallel Huffman decode), feeding jpeg.hip's IDCT / colour kernels.
//
// Replaces the host entropy stage of the frame read (jpeg_host.cpp: cv2.imread of
// the ffmpeg-split frames, combine_detect.py:167-172; libjpeg-turbo's jdhuff.c
// [ext] decode restated). A frame's entropy-coded segment is one sequential bit
// stream (the ffmpeg-split frames carry no restart markers), so it is cut into
// fixed-size chunks of raw bytes, one thread each, and decoded speculatively:
//
//   jdec_prep_kernel   per frame: stuffed 0x00 bytes per chunk, exclusive scan ->
//                      D[i], the data-bit position of chunk i's first byte
//                      (positions count data bits, stuffed bytes excluded).
//   jdec_sync_kernel   chunk i decodes whole blocks (MCU order) from a start state
//                      (data-bit position, block-in-MCU u; a state is always a
//                      block boundary) until the first block boundary at or past
//                      chunk i+1's start: its exit state E[i], blocks started and
//                      the sum of DC differences per component. Pass 0 starts every
//                      chunk at its first data bit with u = 0 (exact for chunk 0);
//                      pass p > 0 restarts chunk i from E[i-1] of pass p-1 where that
//                      differs from the state it last started from. Huffman codes
//                      resynchronise within a few codewords, and the block-in-MCU
//                      phase within a few MCUs (luma and chroma tables differ), so a
//                      wrong start converges onto the true block boundaries and E[i]
//                      stops changing; the host launches passes until no exit state
//                      changes. In speculative passes an invalid code or a run past
//                      the block ends the block (a wrong start must keep going).
//   jdec_scan_kernel   per frame: exclusive scans of the block counts and DC sums
//                      -> each chunk's first block index and DC predictors.
//   jdec_write_kernel  each chunk decodes its blocks once more from its final start
//                      state, DC = predictor + difference, coefficients dequantised
//                      later by jpeg_idct_kernel; blocks go dense (int16 natural
//                      order, component-plane block order) through a per-thread LDS
//                      block; an invalid code or a run past a block here is a
//                      corrupt stream (the frame is rejected, as the host decoder).
// Early stop (option jdec_sync = R > 0): every decode records the first R block-
// boundary states of its trajectory (position, phase, DC sums so far), and a pass-p
// decode that reaches a state of the chunk's previous trajectory stops there: a state
// determines everything after it, so the rest of the decode, its exit state, block
// count and DC sums are the previous ones (counts and sums adjusted by the recorded
// prefix), and the new trajectory's list is the new prefix plus the old suffix. A
// resynchronisation pass then costs the distance to the meeting point rather than a
// whole chunk (noise frames at q95 need 50-200 blocks, 1-5 chunks, to converge from a
// wrong start, so several passes run; real frames a few blocks).
// Tables (jpeg_host.cpp build_huff, per distinct DHT set of the batch): an 11-bit
// lookahead for every table, libjpeg-turbo's AC fast path (code + extra bits in one
// lookup), and the canonical maxcode / valoff / vals slow path for longer codes.
#include "vd_common.h"

namespace {

constexpr int kLook = 11;
constexpr int WG = 256;

__constant__ int kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                             41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                             30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};


// data-bit reader over raw scan bytes: 0xFF 0x00 -> 0xFF, a marker or the end of the
// segment feeds zeros (jdhuff.c fill_bit_buffer). Each lane holds 64 raw bytes of
// its stream in registers ([wb, wb + 64), wb 16-B aligned). Refills are wave-wide:
// refill() runs at the start of every symbol on all active lanes, and when any of
// them has fewer than kLow bytes left, all of them reload 64 bytes from their read
// position -- one memory latency per refill for the whole wave instead of one per
// lane and window (lanes cross their windows at unrelated times, and a wave waits
// for every load any lane issues). A symbol consumes at most one fill: 8 data bytes,
// 16 raw bytes with stuffing, so kLow = 24 keeps every read inside the buffer.
constexpr uint32_t kLow = 24;

struct Reader {
    const uint8_t* d;
    uint32_t n;                // raw bytes of the segment
    uint32_t p;                // next raw byte to fetch
    uint64_t acc;              // left-aligned bit buffer
    int nb;
    bool end;
    uint32_t pos;              // data-bit position of acc's top bit
    uint32_t wb;               // raw byte of w[0]
    uint32_t w[16];

    __device__ __forceinline__ void load(uint32_t base) {
        wb = base;
        const uint4* src = (const uint4*)(d + base);
        const uint4 a0 = src[0], a1 = src[1], a2 = src[2], a3 = src[3];
        w[0] = a0.x; w[1] = a0.y; w[2] = a0.z; w[3] = a0.w;
        w[4] = a1.x; w[5] = a1.y; w[6] = a1.z; w[7] = a1.w;
        w[8] = a2.x; w[9] = a2.y; w[10] = a2.z; w[11] = a2.w;
        w[12] = a3.x; w[13] = a3.y; w[14] = a3.z; w[15] = a3.w;
    }
    // wave-uniform point: every active lane calls it
    __device__ __forceinline__ void refill() {
        const bool low = wb + 64u - p < kLow;
        if (__builtin_amdgcn_ballot_w64(low)) load(p & ~15u);
    }
    __device__ __forceinline__ uint32_t word(uint32_t q) const {   // w[q], q in [0, 16), no dynamic indexing
        const uint32_t b0 = q & 1u, b1 = q & 2u, b2 = q & 4u, b3 = q & 8u;
        const uint32_t l0 = b0 ? w[1] : w[0], l1 = b0 ? w[3] : w[2], l2 = b0 ? w[5] : w[4], l3 = b0 ? w[7] : w[6];
        const uint32_t l4 = b0 ? w[9] : w[8], l5 = b0 ? w[11] : w[10], l6 = b0 ? w[13] : w[12], l7 = b0 ? w[15] : w[14];
        const uint32_t m0 = b1 ? l1 : l0, m1 = b1 ? l3 : l2, m2 = b1 ? l5 : l4, m3 = b1 ? l7 : l6;
        const uint32_t n0 = b2 ? m1 : m0, n1 = b2 ? m3 : m2;
        return b3 ? n1 : n0;
    }
    __device__ __forceinline__ uint32_t byte_at(uint32_t i) const {
        if (i >= n) return 0x100u;                              // past the segment
        const uint32_t o = i - wb;
        return (word(o >> 2) >> ((o & 3u) * 8u)) & 0xFFu;
    }
    // make nb >= 32: four data bytes at once when none is 0xFF (the common case), else
    // byte by byte with the stuffing / marker rules
    __device__ __forceinline__ void topup() {
        if (!end && p + 4u <= n) {
            const uint32_t o = p - wb;
            const uint32_t v = __builtin_amdgcn_alignbyte(word((o >> 2) + 1u), word(o >> 2), o & 3u);
            const uint32_t x = ~v;
            if (((x - 0x01010101u) & ~x & 0x80808080u) == 0u) {   // no 0xFF byte
                const uint32_t be = __builtin_bswap32(v);
                acc |= (uint64_t)be << (32 - nb);
                nb += 32;
                p += 4;
                return;
            }
        }
        while (nb < 32) {
            uint32_t v = 0;
            if (!end) {
                const uint32_t c = byte_at(p);
                if (c > 0xFFu) {
                    end = true;
                } else if (c == 0xFFu) {
                    if (byte_at(p + 1) == 0u) { v = 0xFFu; p += 2; }
                    else end = true;                            // a marker: zeros from here
                } else {
                    v = c;
                    ++p;
                }
            }
            acc |= (uint64_t)v << (56 - nb);
            nb += 8;
        }
    }
    // start of a symbol (wave-uniform point): buffer reload if any lane runs low, then
    // at least 32 bits in acc -- one symbol with its extra bits needs at most 27
    __device__ __forceinline__ void step() {
        refill();
        if (nb < 32) topup();
    }
    // start at raw byte r (whose first data bit is data position dpos), then skip to `to`
    // (wave-uniform: every active lane calls it)
    __device__ void seek(const uint8_t* data, uint32_t nbytes, uint32_t r, uint32_t dpos, uint32_t to) {
        d = data; n = nbytes; p = r; acc = 0; nb = 0; end = false; pos = dpos;
        load(p & ~15u);
        if (p > 0 && p < n && byte_at(p) == 0u && (p - 1 >= wb ? byte_at(p - 1) : (uint32_t)d[p - 1]) == 0xFFu)
            ++p;                                                // a stuffed byte: no data
        uint32_t k = to - dpos;
        while (k) {
            step();
            const int s = k > 32 ? 32 : (int)k;
            acc <<= s; nb -= s; pos += s; k -= s;
        }
    }
    __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(acc >> (64 - k)); }   // after step()
    __device__ __forceinline__ void skip(int k) { acc <<= k; nb -= k; pos += k; }
    __device__ __forceinline__ int get(int k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return (int)v;
    }
};

__device__ __forceinline__ int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

__device__ __forceinline__ int decode_sym(Reader& b, const JLds& T, int t) {
    const uint32_t look = b.peek(kLook);
    const uint32_t e = T.look[t][look];
    if (e >> 8) {
        b.skip((int)(e >> 8));
        return (int)(e & 0xFFu);
    }
    const uint32_t code = b.peek(16);
    for (int len = kLook - 1; len <= 16; ++len) {
        const int c = (int)(code >> (16 - len));
        if (T.maxcode[t][len] >= 0 && c <= T.maxcode[t][len]) {
            b.skip(len);
            return T.vals[t][(T.valoff[t][len] + c) & 255];
        }
    }
    return -1;
}

// per batch
struct JdecArgs {
    const uint8_t* bytes;          // raw scan segments, frame f at bytes + seg_off[f] (16-B aligned)
    const uint32_t* seg_off;       // [n]
    const uint32_t* seg_len;       // [n] raw bytes
    const uint32_t* chunk0;        // [n + 1] first global chunk of each frame
    const uint8_t* tab_of;         // [n] table set per frame
    const JLds* tabs;              // [sets]
    int n, chunk_bytes;
    int bpm;                       // blocks per MCU
    int ucomp[6], udc[6], uac[6];  // per block-in-MCU: component, DC / AC table (0..1 of the set)
    int ubx[6], uby[6];            // its block offset within the MCU's component area
    int mcux, total_blocks;        // per frame
    int cblk[3], bw[3], hs[3], vs[3];
    int blocks_per_image;
    // per chunk
    uint32_t* D;                   // [chunks + frames] data-bit start (frame end at chunk0[f+1] + f)
    uint32_t* stuffed;             // scratch [chunks]
    uint32_t* S;                   // start state: pos
    uint8_t* Su;                   //   block-in-MCU
    uint32_t* Epos[2]; uint8_t* Eu[2];   // exit state, ping-pong per pass
    uint32_t* nblk;                // blocks started
    int* dcs;                      // [chunks][3] DC difference sums
    uint32_t* base;                // first block index (scan)
    int* dcoff;                    // [chunks][3] DC predictors at the chunk start
    int16_t* dense;                // [n][blocks_per_image][64]
    int* flags;                    // [1] corrupt stream; [4 + p] exit states changed in pass p (p <= 64)
    // early stop: the first R states of each chunk's current trajectory, two list buffers
    int R;                         // states recorded per chunk (0: off)
    uint32_t* Lpos[2]; uint8_t* Lu[2];   // [chunks][R]
    int* Ldc[2];                   // [chunks][R][3] DC difference sums before the state
    uint8_t* Lcnt[2];              // [chunks] states in the list
    uint8_t* Lsel;                 // [chunks] buffer holding the chunk's current list
    uint32_t* own;                 // [chunks] blocks the write decodes
};

// one frame per workgroup: stuffed bytes per chunk -> data-bit positions
__global__ __launch_bounds__(WG) void jdec_prep_kernel(JdecArgs a) {
    const int f = blockIdx.x, t = threadIdx.x;
    const uint8_t* d = a.bytes + a.seg_off[f];
    const uint32_t nbytes = a.seg_len[f];
    const uint32_t c0 = a.chunk0[f], nch = a.chunk0[f + 1] - c0;
    __shared__ uint32_t s[WG];
    uint32_t carry = 0;
    for (uint32_t g0 = 0; g0 < nch; g0 += WG) {
        const uint32_t i = g0 + t;
        uint32_t cnt = 0;
        if (i < nch) {   // 0xFF 0x00 pairs whose 0x00 lies in the chunk, 16 bytes at a time
            const uint32_t r0 = i * a.chunk_bytes, r1 = min(nbytes, r0 + a.chunk_bytes);
            uint32_t prev_ff = r0 > 0 && d[r0 - 1] == 0xFFu ? 1u : 0u;   // previous byte is 0xFF
            for (uint32_t r = r0; r < r1; r += 16) {
                const uint4 v = *(const uint4*)(d + r);                  // 16-B aligned (chunk_bytes % 16 == 0)
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
                const uint32_t valid = r1 - r;                          // bytes of this vector in the chunk
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t w = wv[k];
                    // exact per-byte masks (0x80 in each byte that is 0x00 / 0xFF)
                    const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
                    const uint32_t nw = ~w;
                    const uint32_t ff = ~(((nw & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | nw | 0x7F7F7F7Fu);
                    uint32_t pairs = ((ff << 8) | (prev_ff << 7)) & z;           // 0xFF then 0x00
                    const uint32_t nvalid = valid > 4u * k ? min(valid - 4u * k, 4u) : 0u;
                    pairs &= nvalid >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nvalid)) - 1u);
                    cnt += __builtin_popcount(pairs);
                    prev_ff = ff >> 31;
                }
            }
        }
        s[t] = cnt;
        __syncthreads();
        for (int o = 1; o < WG; o <<= 1) {                 // inclusive Hillis-Steele scan
            const uint32_t v = t >= o ? s[t - o] : 0u;
            __syncthreads();
            s[t] += v;
            __syncthreads();
        }
        if (i < nch) a.D[c0 + f + i] = 8u * (i * (uint32_t)a.chunk_bytes - (carry + s[t] - cnt));
        carry += s[WG - 1];
        __syncthreads();
    }
    if (t == 0) a.D[c0 + f + nch] = 8u * (nbytes - carry);   // the frame's data bits (chunk end of the last)
}

// Per-lane symbol loop (one symbol of every lane per iteration: DC and AC symbols
// share the table lookup, so lanes in different coefficient positions do not split
// the wave into separate DC / AC paths). Block boundaries (k == 0) are where a decode
// stops, records its state or meets an earlier trajectory.
//   MODE 0: count until the first boundary at or past `stop` (speculative: an invalid
//           code or a run past the block ends the block, a wrong start keeps going)
//   MODE 2: MODE 0, recording the first R states into list 0
//   MODE 3: MODE 0, recording into list `nxt` and stopping at a state of list `cur`
//   MODE 1: write exactly `limit` blocks (the first at global block blk0) straight
//           into the zeroed dense buffer; an invalid code or a run past the block is a
//           corrupt stream (bad)
struct Walk {
    uint32_t stop, limit, blk0;
    size_t L0;
    int cur, nxt;                  // MODE 3 lists
    uint32_t cnt, j;               // MODE 3: cur list length, merge index (in/out)
    int16_t* dense;                // MODE 1: the frame's dense blocks
    bool met, bad;
};

__device__ __forceinline__ void record(const JdecArgs& a, int buf, size_t at, uint32_t pos, int u, const int (&dcs)[3]) {
    uint32_t* lp = buf ? a.Lpos[1] : a.Lpos[0];
    uint8_t* lu = buf ? a.Lu[1] : a.Lu[0];
    int* ld = buf ? a.Ldc[1] : a.Ldc[0];
    lp[at] = pos;
    lu[at] = (uint8_t)u;
    ld[at * 3] = dcs[0];
    ld[at * 3 + 1] = dcs[1];
    ld[at * 3 + 2] = dcs[2];
}

template <int MODE>
__device__ __forceinline__ void decode_run(const JdecArgs& a, const JLds& T, Reader& b, int& u, uint32_t& nblk,
                                           int (&dcs)[3], int (&pred)[3], Walk& w, const uint8_t* zig = nullptr) {
    // per block-in-MCU tables / component as packed bit fields (no per-lane indexing of kernel arguments)
    uint32_t pk_c = 0, pk_dc = 0, pk_ac = 0, pk_bx = 0, pk_by = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        pk_c |= (uint32_t)a.ucomp[i] << (2 * i);
        pk_dc |= (uint32_t)(a.udc[i] & 1) << i;
        pk_ac |= (uint32_t)(a.uac[i] & 1) << i;
        pk_bx |= (uint32_t)(a.ubx[i] & 1) << i;
        pk_by |= (uint32_t)(a.uby[i] & 1) << i;
    }
    const uint32_t* dcop = MODE == 3 ? (w.cur ? a.Lpos[1] : a.Lpos[0]) + w.L0 : nullptr;
    const uint8_t* dcou = MODE == 3 ? (w.cur ? a.Lu[1] : a.Lu[0]) + w.L0 : nullptr;
    // MODE 3: entries j and j+1 of the previous trajectory in registers, the next one
    // loaded a block ahead of its use (a dependent global load per boundary otherwise)
    uint32_t p0 = 0xFFFFFFFFu, p1 = 0xFFFFFFFFu, u0 = 0, u1 = 0;
    if constexpr (MODE == 3) {
        if (w.j < w.cnt) { p0 = dcop[w.j]; u0 = dcou[w.j]; }
        if (w.j + 1 < w.cnt) { p1 = dcop[w.j + 1]; u1 = dcou[w.j + 1]; }
    }
    int k = 0, c = 0, tdc = 0, tac = 0;
    int16_t* dst = nullptr;
    for (;;) {
        if (k == 0) {                                           // block boundary
            bool live = MODE == 1 ? (nblk < w.limit && w.blk0 + nblk < (uint32_t)a.total_blocks) : b.pos < w.stop;
            if constexpr (MODE == 3) {
                if (live) {
                    while (w.j < w.cnt && p0 < b.pos) {             // advance: usually one step, prefetched
                        ++w.j;
                        p0 = p1; u0 = u1;
                        if (w.j + 1 < w.cnt) { p1 = dcop[w.j + 1]; u1 = dcou[w.j + 1]; }
                        else p1 = 0xFFFFFFFFu;
                    }
                    if (w.j < w.cnt && p0 == b.pos && u0 == (uint32_t)u) { w.met = true; live = false; }
                }
            }
            if (!live) break;
            if constexpr (MODE == 2 || MODE == 3) {
                if (nblk < (uint32_t)a.R) record(a, MODE == 2 ? 0 : w.nxt, w.L0 + nblk, b.pos, u, dcs);
            }
            c = (int)((pk_c >> (2 * u)) & 3u);
            tdc = (int)((pk_dc >> u) & 1u);
            tac = (int)((pk_ac >> u) & 1u);
            if constexpr (MODE == 1) {
                const uint32_t g = w.blk0 + nblk;
                const uint32_t m = g / a.bpm;
                const int mx = (int)(m % a.mcux), my = (int)(m / a.mcux);
                const int bx = (int)((pk_bx >> u) & 1u), by = (int)((pk_by >> u) & 1u);
                const size_t pb = (size_t)a.cblk[c] + (size_t)(my * a.vs[c] + by) * a.bw[c] + mx * a.hs[c] + bx;
                dst = w.dense + pb * 64;
            }
        }
        b.step();
        const uint32_t look = b.peek(kLook);
        const bool isdc = k == 0;
        const uint32_t* tb = isdc ? T.fastdc[tdc] : T.fast[tac];
        const uint32_t e = tb[look];
        int run, val;
        if (e & 0xFFu) {
            b.skip((int)(e & 0xFFu));
            run = (int)((e >> 8) & 0xFFu);
            val = (int)(int16_t)(e >> 16);
        } else {                                                // code + extra bits longer than the lookahead
            int rs = decode_sym(b, T, isdc ? tdc : 2 + tac);
            if (isdc) {
                if (rs < 0 || rs > 11) {
                    if constexpr (MODE == 1) { w.bad = true; return; }
                    if (rs < 0) b.skip(1);                      // keep moving: a wrong start resyncs
                    rs = 0;
                }
                run = 0;
                val = extend(b.get(rs), rs);
            } else if (rs < 0) {
                if constexpr (MODE == 1) { w.bad = true; return; }
                b.skip(1);
                run = 64;                                       // the block ends
                val = 0;
            } else {
                const int r = rs >> 4, sz = rs & 15;
                run = sz == 0 ? (r == 15 ? 16 : 64) : r;
                val = sz == 0 ? 0 : extend(b.get(sz), sz);
            }
        }
        if (isdc) {
            dcs[0] += c == 0 ? val : 0;
            dcs[1] += c == 1 ? val : 0;
            dcs[2] += c == 2 ? val : 0;
            if constexpr (MODE == 1) {
                pred[0] += c == 0 ? val : 0;
                pred[1] += c == 1 ? val : 0;
                pred[2] += c == 2 ? val : 0;
                dst[0] = (int16_t)(c == 0 ? pred[0] : (c == 1 ? pred[1] : pred[2]));
            }
            k = 1;
        } else if (run == 64) {                                 // EOB
            k = 64;
        } else if (run == 16) {                                 // ZRL (a coefficient's run is <= 15)
            k += 16;
        } else {
            k += run;
            if (k > 63) {
                if constexpr (MODE == 1) { w.bad = true; return; }
                k = 64;
            } else {
                if constexpr (MODE == 1) dst[zig[k]] = (int16_t)val;
                ++k;
            }
        }
        if (k >= 64) {                                          // the block is done
            ++nblk;
            u = u + 1 == a.bpm ? 0 : u + 1;
            k = 0;
        }
    }
}

__device__ __forceinline__ void load_tables(const JdecArgs& a, int f, JLds* T) {
    const uint32_t* src = (const uint32_t*)(a.tabs + a.tab_of[f]);
    uint32_t* dst = (uint32_t*)T;
    for (int i = threadIdx.x; i < (int)(sizeof(JLds) / 4); i += WG) dst[i] = src[i];
    __syncthreads();
}

// pass 0 (first = 1) or a resynchronisation pass over every chunk of the batch;
// workgroups never straddle frames (wg_frame / wg_chunk0 from the host)
__global__ __launch_bounds__(WG) void jdec_sync_kernel(JdecArgs a, const int* wg_frame, const uint32_t* wg_chunk,
                                                        int pass) {
    __shared__ JLds T;
    const int f = wg_frame[blockIdx.x];
    load_tables(a, f, &T);
    const uint32_t c0 = a.chunk0[f], nch = a.chunk0[f + 1] - c0;
    const uint32_t i = wg_chunk[blockIdx.x] + threadIdx.x;        // chunk within the frame
    if (i >= nch) return;
    const uint32_t g = c0 + i;
    const int pi = (pass + 1) & 1, po = pass & 1;                  // pass p reads E[(p-1)&1], writes E[p&1]
    uint32_t spos;
    int su;
    if (pass == 0) {
        spos = a.D[c0 + f + i];
        su = 0;
    } else {
        if (i == 0) {                                             // exact since pass 0
            a.Epos[po][g] = a.Epos[pi][g];
            a.Eu[po][g] = a.Eu[pi][g];
            return;
        }
        spos = a.Epos[pi][g - 1];
        su = a.Eu[pi][g - 1];
        if (spos == a.S[g] && su == a.Su[g]) {                    // same start: same decode
            a.Epos[po][g] = a.Epos[pi][g];
            a.Eu[po][g] = a.Eu[pi][g];
            return;
        }
    }
    Reader b;
    b.seek(a.bytes + a.seg_off[f], a.seg_len[f], i * (uint32_t)a.chunk_bytes, a.D[c0 + f + i], spos);
    int u = su;
    uint32_t nb = 0;
    int dcs[3] = {0, 0, 0}, pred[3] = {0, 0, 0};
    const size_t L0 = (size_t)g * a.R;
    Walk w{};
    w.stop = a.D[c0 + f + i + 1];
    w.L0 = L0;
    if (a.R == 0) {
        decode_run<0>(a, T, b, u, nb, dcs, pred, w);
    } else if (pass == 0) {
        decode_run<2>(a, T, b, u, nb, dcs, pred, w);
        a.Lcnt[0][g] = (uint8_t)min(nb, (uint32_t)a.R);
        a.Lsel[g] = 0;
    } else {
        // decode until the chunk's end or a state of its previous trajectory
        const int cur = a.Lsel[g], nxt = cur ^ 1;
        const uint32_t cnt = a.Lcnt[cur][g];
        const uint32_t* op = a.Lpos[cur] + L0;
        const uint8_t* ou = a.Lu[cur] + L0;
        w.cur = cur; w.nxt = nxt; w.cnt = cnt; w.j = 0;
        decode_run<3>(a, T, b, u, nb, dcs, pred, w);
        const bool met = w.met;
        const uint32_t j = w.j;
        uint32_t ncnt = min(nb, (uint32_t)a.R);
        if (met) {   // the rest is the previous decode: its suffix, exit state and sums
            const int* od = a.Ldc[cur] + L0 * 3;
            int dm[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) dm[c] = od[j * 3 + c];
            for (uint32_t t = j; t < cnt && nb + (t - j) < (uint32_t)a.R; ++t) {
                const uint32_t q = nb + (t - j);
                a.Lpos[nxt][L0 + q] = op[t];
                a.Lu[nxt][L0 + q] = ou[t];
#pragma unroll
                for (int c = 0; c < 3; ++c) a.Ldc[nxt][(L0 + q) * 3 + c] = dcs[c] + od[t * 3 + c] - dm[c];
                ncnt = q + 1;
            }
            const uint32_t nb_old = a.nblk[g];
            a.nblk[g] = nb + (nb_old - j);
#pragma unroll
            for (int c = 0; c < 3; ++c) a.dcs[(size_t)g * 3 + c] = dcs[c] + a.dcs[(size_t)g * 3 + c] - dm[c];
            a.Lcnt[nxt][g] = (uint8_t)ncnt;
            a.Lsel[g] = (uint8_t)nxt;
            a.S[g] = spos;
            a.Su[g] = (uint8_t)su;
            a.Epos[po][g] = a.Epos[pi][g];
            a.Eu[po][g] = a.Eu[pi][g];
            return;
        }
        a.Lcnt[nxt][g] = (uint8_t)ncnt;
        a.Lsel[g] = (uint8_t)nxt;
    }
    a.S[g] = spos;
    a.Su[g] = (uint8_t)su;
    a.nblk[g] = nb;
#pragma unroll
    for (int c = 0; c < 3; ++c) a.dcs[(size_t)g * 3 + c] = dcs[c];
    if (pass > 0 && (b.pos != a.Epos[pi][g] || (uint8_t)u != a.Eu[pi][g])) atomicOr(a.flags + 4 + pass, 1);
    a.Epos[po][g] = b.pos;
    a.Eu[po][g] = (uint8_t)u;
}

// per frame: exclusive scans of block counts and DC sums over its chunks
__global__ __launch_bounds__(WG) void jdec_scan_kernel(JdecArgs a) {
    const int f = blockIdx.x, t = threadIdx.x;
    const uint32_t c0 = a.chunk0[f], nch = a.chunk0[f + 1] - c0;
    __shared__ int s[4][WG];
    int carry[4] = {0, 0, 0, 0};
    for (uint32_t g0 = 0; g0 < nch; g0 += WG) {
        const uint32_t i = g0 + t;
        int v[4] = {0, 0, 0, 0};
        if (i < nch) {
            const uint32_t g = c0 + i;
            v[0] = (int)a.nblk[g];
            for (int c = 0; c < 3; ++c) v[1 + c] = a.dcs[(size_t)g * 3 + c];
            a.own[g] = (uint32_t)v[0];
        }
        for (int q = 0; q < 4; ++q) s[q][t] = v[q];
        __syncthreads();
        for (int o = 1; o < WG; o <<= 1) {
            int x[4];
            for (int q = 0; q < 4; ++q) x[q] = t >= o ? s[q][t - o] : 0;
            __syncthreads();
            for (int q = 0; q < 4; ++q) s[q][t] += x[q];
            __syncthreads();
        }
        if (i < nch) {
            a.base[c0 + i] = (uint32_t)(carry[0] + s[0][t] - v[0]);
            for (int c = 0; c < 3; ++c) a.dcoff[(size_t)(c0 + i) * 3 + c] = carry[1 + c] + s[1 + c][t] - v[1 + c];
        }
        for (int q = 0; q < 4; ++q) carry[q] += s[q][WG - 1];
        __syncthreads();
    }
}

__global__ __launch_bounds__(WG) void jdec_write_kernel(JdecArgs a, const int* wg_frame, const uint32_t* wg_chunk) {
    __shared__ JLds T;
    __shared__ uint8_t zig[64];                                    // zigzag -> natural (LDS: a per-lane index)
    if (threadIdx.x < 64) zig[threadIdx.x] = (uint8_t)kZig[threadIdx.x];
    const int f = wg_frame[blockIdx.x];
    load_tables(a, f, &T);
    const uint32_t c0 = a.chunk0[f], nch = a.chunk0[f + 1] - c0;
    const uint32_t i = wg_chunk[blockIdx.x] + threadIdx.x;
    if (i >= nch) return;
    const uint32_t g = c0 + i;
    Reader b;
    b.seek(a.bytes + a.seg_off[f], a.seg_len[f], i * (uint32_t)a.chunk_bytes, a.D[c0 + f + i], a.S[g]);
    int u = a.Su[g];
    uint32_t nb = 0;
    int dcs[3] = {0, 0, 0};
    int pred[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) pred[c] = a.dcoff[(size_t)g * 3 + c];
    Walk w{};
    w.limit = a.own[g];
    w.blk0 = a.base[g];
    w.dense = a.dense + (size_t)f * a.blocks_per_image * 64;
    decode_run<1>(a, T, b, u, nb, dcs, pred, w, zig);
    const bool bad = w.bad;
    if (bad) atomicOr(a.flags + 1, 1);
    if (i + 1 == nch && a.base[g] + nb < (uint32_t)a.total_blocks) atomicOr(a.flags + 1, 2);   // too few blocks
}

}  // namespace

// one stage of the device entropy decode (jpeg_host.cpp drives the sequence)
hipError_t vd_launch_jdec(const JdecLaunch& L, hipStream_t s) {
    JdecArgs a{};
    a.bytes = L.bytes; a.seg_off = L.seg_off; a.seg_len = L.seg_len; a.chunk0 = L.chunk0; a.tab_of = L.tab_of;
    a.tabs = (const JLds*)L.tabs; a.n = L.n; a.chunk_bytes = L.chunk_bytes; a.bpm = L.bpm;
    for (int k = 0; k < 6; ++k) { a.ucomp[k] = L.ucomp[k]; a.udc[k] = L.udc[k]; a.uac[k] = L.uac[k]; a.ubx[k] = L.ubx[k]; a.uby[k] = L.uby[k]; }
    a.mcux = L.mcux; a.total_blocks = L.total_blocks;
    for (int c = 0; c < 3; ++c) { a.cblk[c] = L.cblk[c]; a.bw[c] = L.bw[c]; a.hs[c] = L.hs[c]; a.vs[c] = L.vs[c]; }
    a.blocks_per_image = L.blocks_per_image;
    a.D = L.D; a.stuffed = nullptr; a.S = L.S; a.Su = L.Su;
    a.Epos[0] = L.Epos[0]; a.Epos[1] = L.Epos[1]; a.Eu[0] = L.Eu[0]; a.Eu[1] = L.Eu[1];
    a.nblk = L.nblk; a.dcs = L.dcs; a.base = L.base; a.dcoff = L.dcoff; a.dense = L.dense; a.flags = L.flags;
    a.R = L.R; a.Lsel = L.Lsel; a.own = L.own;
    for (int k = 0; k < 2; ++k) { a.Lpos[k] = L.Lpos[k]; a.Lu[k] = L.Lu[k]; a.Ldc[k] = L.Ldc[k]; a.Lcnt[k] = L.Lcnt[k]; }
    if (L.stage == 0) {
        hipLaunchKernelGGL(jdec_prep_kernel, dim3(a.n), dim3(WG), 0, s, a);
    } else if (L.stage == 1) {
        hipLaunchKernelGGL(jdec_sync_kernel, dim3(L.nwg), dim3(WG), 0, s, a, L.wg_frame, L.wg_chunk, L.pass);
    } else if (L.stage == 2) {
        hipLaunchKernelGGL(jdec_scan_kernel, dim3(a.n), dim3(WG), 0, s, a);
    } else {
        hipLaunchKernelGGL(jdec_write_kernel, dim3(L.nwg), dim3(WG), 0, s, a, L.wg_frame, L.wg_chunk);
    }
    return hipGetLastError();
}
