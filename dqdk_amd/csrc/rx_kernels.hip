/*
 * rx_kernels.hip -- gfx950 kernels of the DQDK receive hot path.
 * See rx_kernels.h for the kernel map and DESIGN.md for the data layout and
 * the roofline each kernel is measured against.
 */
#include "rx_kernels.h"

namespace dqdk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// (a helper taking the dword by value: __builtin_bit_cast applied directly
// to an ext_vector element such as v.y reads element 0 with hipcc 7.2)
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ u32x2 as_u32x2(uint64_t x) { return __builtin_bit_cast(u32x2, x); }
__device__ __forceinline__ u32x4 as_u32x4(u64x2 x) { return __builtin_bit_cast(u32x4, x); }

// Byte layout constants (src/tristan.h:55-60).
constexpr uint32_t kChannels = DQDK_TRISTAN_CHANNELS;
constexpr uint32_t kHists = DQDK_TRISTAN_HISTS;

// Streaming geometry of one frame, relative to a0 = frame address & ~15.
// Chunk c covers bytes [16c + q4, 16c + q4 + 16): q4 puts event byte 2 of
// every event at a fixed dword (offset r) of one chunk, so a lane decodes an
// event from its own 16 B (no cross-lane shuffles).  Phase B streams chunks
// [c_begin, c_begin + nch) as 2-KiB windows, 32 B (two chunks) per lane.
struct Geo {
    int q4, r;       // grid shift; byte offset of event byte 2 in its chunk
    int c_begin;     // first streamed chunk
    int nch;         // streamed chunks
    int nwin;        // 2-KiB windows (128 chunks)
    int de;          // chunk of event 0, relative to c_begin (-7..1: negative when phase A took events)
    int ct;          // last checksum chunk relative to c_begin (-1: no checksum bytes streamed)
    int keep;        // checksum bytes in chunk ct (1..16)
    int cs_lo;       // checksum start (a0-relative): bytes [16 c_begin + q4, cs_lo) are the head correction
    int cs_hi;       // checksum end (a0-relative, the odd-length over-read byte included)
};

constexpr int kLaneBytes = 32;                    // two chunks per lane per window
constexpr int kWinChunks = 64 * kLaneBytes / 16;  // 128
constexpr uint32_t kWinBytes = 64u * kLaneBytes;  // 2 KiB

//
// a_end > 0 (the fused decode at 1500 B): phase A, which read the frame's
// first cache line [0, a_end) already, decodes every event whose chunk ends
// inside it and sums the checksum bytes before the chunk holding byte a_end;
// the stream starts at that chunk, so phase B re-reads no more of that line
// than its last chunk's head.
__device__ __forceinline__ Geo frame_geo(uint32_t work, uint32_t off0, uint32_t poff, uint32_t hs, uint32_t len16,
                                         uint32_t E, int a_end = 0)
{
    Geo g;
    const bool dec = work & 1, cs = work & 2;
    const int dec_lo = (int)(off0 + poff);
    const int dec_hi = dec_lo + (int)(16 * E);
    const int cs_lo = (int)(off0 + 14 + hs);
    const int cs_hi = cs_lo + (int)len16 + (int)(len16 & 1);  // + the odd-length over-read byte
    const int q = dec ? ((dec_lo + 2) & ~3) : 0;
    g.q4 = q & 15;
    g.r = (dec_lo + 2) & 3;
    g.cs_lo = cs_lo;
    g.cs_hi = cs_hi;
    int lo = 0x7fffffff, hi = 0;
    if (dec) {
        lo = dec_lo;
        hi = dec_hi;
    }
    if (cs) {
        lo = min(lo, cs_lo);
        hi = max(hi, cs_hi);
    }
    if (hi <= lo) {
        g.c_begin = g.nch = g.nwin = g.de = g.keep = 0;
        g.ct = -1;
        return g;
    }
    g.c_begin = (lo - g.q4) >> 4;  // lo >= 14 > q4
    if (a_end > 0)
        g.c_begin = max(g.c_begin, (a_end - g.q4) >> 4);  // (a_end >= 16 > q4)
    g.nch = max(((hi - g.q4 + 15) >> 4) - g.c_begin, 0);
    g.nwin = (g.nch + kWinChunks - 1) / kWinChunks;
    // 0 or 1 (the chunk of event byte 2 is c_begin or the next); negative:
    // phase A decoded -de events
    g.de = dec ? (q >> 4) - g.c_begin : 0;
    const int ct = (cs_hi - 1 - g.q4) >> 4;
    if (cs && cs_hi > cs_lo && ct >= g.c_begin) {
        g.ct = ct - g.c_begin;
        g.keep = cs_hi - (16 * ct + g.q4);
    } else {
        g.ct = -1;
        g.keep = 16;
    }
    return g;
}

// Per-frame hand-off from phase A (lane per frame) to phase B (wave per frame).
struct FrameInfo {
    uint64_t addr;     // (phase A only: phase C re-reads the descriptor for the write-back)
    uint32_t pseudo;   // saddr + daddr + ((17 + len16) << 8), the csum_tcpudp_nofold terms, folded to
                       //   32 bits (end-around carry: the same value mod 0xffff, all the verdict uses)
    uint8_t odd;       // the UDP header starts at an odd address
    uint32_t datalen;
    uint16_t len16;    // (u16)udplen handed to udp_audit_checksum
    uint16_t check;    // udp->check as stored (LE u16)
    uint8_t status;
    uint8_t poff;      // payload offset from the frame start
    uint8_t work;      // bit0 decode, bit1 udp checksum pending
    uint8_t hs;        // ihl * 4
    uint32_t head;     // checksum head correction: word sum of bytes [16 c_begin + q4, cs_lo)
    Geo g;
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int b) { return (w >> (8 * b)) & 0xffu; }

__device__ __forceinline__ uint32_t sel4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t q)
{
    uint32_t lo = (q & 1) ? b : a;
    uint32_t hi = (q & 1) ? d : c;
    return (q & 2) ? hi : lo;
}

// bytes at rel. offset [lo, hi) of a dword starting at rel. offset p -> mask
// Sums of the even- and odd-position bytes [from, to) (0 <= from <= to <= 16)
// of one 16-B chunk held in wave-uniform registers (scalar ALU).
__device__ __forceinline__ void chunk_range_sums(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, int from, int to,
                                                 uint32_t& e, uint32_t& o)
{
    auto below = [](int nbytes) -> uint64_t {
        return nbytes <= 0 ? 0ull : nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1);
    };
    const uint64_t lo = ((uint64_t)x0 | ((uint64_t)x1 << 32)) & (below(to) & ~below(from));
    const uint64_t hi = ((uint64_t)x2 | ((uint64_t)x3 << 32)) & (below(to - 8) & ~below(from - 8));
    const uint64_t M = 0x00ff00ff00ff00ffull;
    uint64_t se = (lo & M) + (hi & M), so = ((lo >> 8) & M) + ((hi >> 8) & M);
    se += se >> 32;
    so += so >> 32;
    e = (uint32_t)(se & 0xffffu) + (uint32_t)((se >> 16) & 0xffffu);
    o = (uint32_t)(so & 0xffffu) + (uint32_t)((so >> 16) & 0xffffu);
}


// Events phase A decodes from the frame's first line (kHeadA): at most 7
// (event 0's chunk starts at or after a0-relative byte 24, the line ends by 128).
constexpr int kAEv = 7;

// Word sum (LE u16 at even a0-relative addresses) of the bytes [lo, hi) of
// the 128 B staged from a0.
__device__ __forceinline__ uint32_t staged_range_sum(const uint32_t (&w)[32], int lo, int hi)
{
    auto below = [](int n) -> uint32_t { return n <= 0 ? 0u : n >= 4 ? 0xffffffffu : ((1u << (8 * n)) - 1u); };
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) {
        const uint32_t m = below(hi - 4 * k) & ~below(lo - 4 * k);
        s = __builtin_amdgcn_udot2(as_u16x2(w[k] & m), u16x2{1, 1}, s, false);
    }
    return s;
}

// ---------------------------------------------------------------------------
// Phase A: one lane parses one frame's headers from 128 B staged in VGPRs.
// kHeadA: it also decodes the events and sums the checksum bytes of the
// frame's first cache line (frame_geo's a_end) into akey[0, na) / fi.head.
// ---------------------------------------------------------------------------
// kHalf: the frame's second 64 B are read only when its headers reach them
// (the records-path tiles: rx_decode, rx_small; r06r: configs[1]'s decode
// -2 %, the fused decode unchanged, so it keeps one 128-B read)
template <bool kHeadA, bool kHalf>
__device__ __forceinline__ void parse_frame(const RxArgs& a, uint32_t i, FrameInfo& fi, dqdk_gpu_rx_result_t& r,
                                            bool& needB, uint32_t (&akey)[kAEv], uint32_t& na, uint32_t& hw, bool& sh)
{
    dqdk_gpu_desc_t d = a.desc[i];
    const uint64_t addr = d.addr;
    const uint32_t len = d.len;
    const uint64_t a0 = addr & ~15ull;
    const uint32_t off0 = (uint32_t)(addr & 15);
    na = 0;
    hw = 0;
    sh = false;

    // 8 aligned chunks = 128 B from a0: covers frame bytes [0, 113) for any off0
    // (the headers need [0, 97)).
    uint32_t w[32];
    auto ld = [&](int k, bool on) {
        u32x4 v = {0u, 0u, 0u, 0u};
        uint64_t o = a0 + 16ull * k;
        if (on && addr < a.umem_size && o + 16 <= a.umem_size)
            v = *(const u32x4*)(a.umem + o);
        w[4 * k + 0] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    };
#pragma unroll
    for (int k = 0; k < 4; k++)
        ld(k, true);
    // The second 64 B only where the parse reads them: without kHeadA it
    // reads a0-relative bytes below off0 + 22 + 4 ihl (prefilter fields,
    // IPv4 header, UDP header, the head correction's bytes before it), so a
    // frame whose headers end inside the first 64 B leaves those bytes 0
    // (ihl = FB(14) & 15: byte 2 of frame dword 3, from w[3..7])
    bool more = true;
    if (kHalf && !kHeadA) {
        const uint32_t q0 = off0 >> 2, rb0 = off0 & 3;
        const uint32_t d3 = __builtin_amdgcn_alignbyte(sel4(w[4], w[5], w[6], w[7], q0),
                                                       sel4(w[3], w[4], w[5], w[6], q0), rb0);
        more = off0 + 22u + 4u * ((d3 >> 16) & 15u) > 64u;
    }
#pragma unroll
    for (int k = 4; k < 8; k++)
        ld(k, more);
    // h[m] = frame dword m (frame-relative, unaligned-safe): static indices below.
    const uint32_t q = off0 >> 2, rb = off0 & 3;
    uint32_t s[22], h[21];
#pragma unroll
    for (int m = 0; m < 22; m++)
        s[m] = sel4(w[m], w[m + 1], w[m + 2], w[m + 3], q);
#pragma unroll
    for (int m = 0; m < 21; m++)
        h[m] = __builtin_amdgcn_alignbyte(s[m + 1], s[m], rb);

#define FB(k) byte_of(h[(k) >> 2], (k) & 3)
    r.datalen = 0;
    r.status = DQDK_RX_OK;
    r.payload_off = 0;
    r.oob_events = 0;
    fi.addr = addr;
    fi.pseudo = 0;
    fi.odd = 0;
    fi.datalen = 0;
    fi.len16 = 0;
    fi.check = 0;
    fi.poff = 0;
    fi.work = 0;
    fi.hs = 0;
    fi.head = 0;
    fi.g = frame_geo(0, 0, 0, 0, 0, 0);
    needB = false;

    if (a.flags & DQDK_GPU_F_PREFILTER) {  // src/bpf/forwarder.bpf.c:38-96
        uint32_t verdict = 2;
        uint32_t sport = (FB(34) << 8) | FB(35);
        if (len <= 14)
            verdict = 0;
        else if (!(FB(12) == 0x08 && FB(13) == 0x00))
            verdict = 1;
        else if (len <= 34)
            verdict = 0;
        else if (FB(23) != 17)
            verdict = 1;
        else if (len <= 42)
            verdict = 0;
        else if (!(sport <= a.port_end && sport >= a.port_start))
            verdict = 1;
        if (verdict != 2) {
            r.status = verdict == 0 ? DQDK_RX_FILTER_DROP : DQDK_RX_FILTER_PASS;
            fi.status = r.status;
            return;
        }
    }

    // get_udp_payload, src/dqdk.c:185-207
    const uint32_t tot_len = (FB(16) << 8) | FB(17);
    const uint32_t ihl = FB(14) & 0xf;
    const uint32_t hs = ihl * 4;
    fi.hs = (uint8_t)hs;
    const bool ip_ok = tot_len == ((len - 14) & 0xffffu);  // ip4_audit (u16)(len-14)
    if (!ip_ok) {
        r.status = DQDK_RX_INVALID_IP;
        fi.status = r.status;
        return;
    }
    if (a.flags & DQDK_GPU_F_CSUM) {
        // ip4_audit_checksum: ~inet_csum(copy with check = 0, ihl*4) on a
        // 4-aligned buffer -- the carry loop of inet_csum.c:92-106.
        uint32_t res = 0, carry = 0;
#pragma unroll
        for (int k = 0; k < 15; k++) {
            uint32_t wk = (h[3 + k] >> 16) | (h[4 + k] << 16);  // IP bytes 4k..4k+3
            if (k == 2)
                wk &= 0x0000ffffu;                           // check field zeroed
            if ((uint32_t)k < ihl) {
                res += carry;
                res += wk;
                carry = wk > res;
            }
        }
        if (ihl >= 1) {
            res += carry;
            res = (res & 0xffff) + (res >> 16);
        }
        res = (res & 0xffff) + (res >> 16);  // from32to16
        res = (res & 0xffff) + (res >> 16);
        const uint32_t calc = (~res) & 0xffffu;
        const uint32_t stored = FB(24) | (FB(25) << 8);
        if (calc != stored) {
            r.status = DQDK_RX_INVALID_IP_CSUM;
            fi.status = r.status;
            return;
        }
    }
    const uint32_t udplen = tot_len - hs;  // u32, may wrap (dqdk.c:197)
    // UDP header at frame byte 14 + hs: dwords 3+ihl.. with a 2-byte shift.
    uint32_t hu1 = 0, hu2 = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if ((uint32_t)k == ihl) {
            hu1 = h[4 + k];
            hu2 = h[5 + k];
        }
    }
    const uint32_t u47 = (hu1 >> 16) | (hu2 << 16);  // udp bytes 4..7
    const uint32_t ulen = ((u47 & 0xff) << 8) | ((u47 >> 8) & 0xff);
    const uint32_t ucheck = u47 >> 16;
    if (ulen != (udplen & 0xffffu)) {  // udp_audit
        r.status = DQDK_RX_INVALID_UDP;
        fi.status = r.status;
        return;
    }
    const uint32_t datalen = udplen - 8;  // dqdk.c:205
    r.datalen = datalen;
    r.payload_off = (uint8_t)(14 + hs + 8);
    r.status = datalen ? DQDK_RX_OK : DQDK_RX_EMPTY;
    fi.status = r.status;
    fi.datalen = datalen;
    fi.poff = r.payload_off;
    const bool pending = (a.flags & DQDK_GPU_F_CSUM) && ucheck != 0;  // udp.c:12-14
    if (pending) {
        const uint32_t saddr = (h[6] >> 16) | (h[7] << 16);
        const uint32_t daddr = (h[7] >> 16) | (h[8] << 16);
        const uint32_t len16 = udplen & 0xffffu;
        fi.len16 = (uint16_t)len16;
        fi.check = (uint16_t)ucheck;
        uint64_t ps = (uint64_t)saddr + (uint64_t)daddr + (uint64_t)(uint32_t)((17u + len16) << 8);
        ps = (ps & 0xffffffffull) + (ps >> 32);  // from64to32 (2^32 = 1 mod 0xffff)
        ps = (ps & 0xffffffffull) + (ps >> 32);
        fi.pseudo = (uint32_t)ps;
        fi.odd = (uint8_t)((addr + 14 + hs) & 1);
        fi.work |= 2;
    }
    // events are decoded only for a consumer: the histogram (histo_fd > 0,
    // src/tristan.c:312) or a caller record buffer
    if (datalen != 0 && a.E != 0 && (a.histo || a.keys))
        fi.work |= 1;
    needB = fi.work != 0;
    if (needB) {
        // phase A takes the first line only when all of it lies inside the
        // UMEM (the bytes it reads are then exactly the stream's)
        const int a_end = kHeadA && a0 + 128 <= a.umem_size ? 128 - (int)(a0 & 127) : 0;
        fi.g = frame_geo(fi.work, off0, fi.poff, hs, fi.len16, a.E, a_end);
        if (kHeadA && a_end > 0 && fi.g.nch > 0) {
            // The stream's first chunk may begin up to 12 B before the line
            // ends (the chunk grid is the events'): phase B would then fetch
            // the whole line again for those bytes (the L2 fetches 128-B
            // lines).  One such dword comes from here instead (sh: lane 0 of
            // the frame's first window loads 4 B further and shifts this dword
            // in); with more, the frame keeps the round-3 geometry.
            const int G0 = 16 * fi.g.c_begin + fi.g.q4;
            if (G0 < a_end) {
                // (the dword travels in LaneFrame::ct, unused unless chunks past
                // the checksum are streamed: such frames keep the old geometry)
                const bool lw = (fi.work & 2) && fi.g.ct < fi.g.nch - 1;
                if (a_end - G0 == 4 && !lw && fi.g.nch >= 2 && a0 + (uint64_t)G0 + 20 <= a.umem_size) {
                    sh = true;
                    // the dword at G0 = a_end - 4: w[31 - 4m], m = (a0 & 127) / 16
                    // (a select tree: a compare-select over all 32 registers
                    // had the compiler emit 8K more instructions in phase A)
                    const uint32_t m = (uint32_t)(a0 & 127) >> 4;
                    const uint32_t h01 = (m & 1) ? w[27] : w[31], h23 = (m & 1) ? w[19] : w[23];
                    const uint32_t h45 = (m & 1) ? w[11] : w[15], h67 = (m & 1) ? w[3] : w[7];
                    const uint32_t h03 = (m & 2) ? h23 : h01, h47 = (m & 2) ? h67 : h45;
                    hw = (m & 4) ? h47 : h03;
                } else {
                    fi.g = frame_geo(fi.work, off0, fi.poff, hs, fi.len16, a.E, 0);
                }
            }
        }
        const int G = 16 * fi.g.c_begin + fi.g.q4;  // the stream's first byte
        const int Lc = fi.g.cs_lo;
        if ((fi.work & 2) && G <= Lc && fi.g.ct >= 0) {
            // head correction: the first streamed chunk starts at G <= cs_lo
            // (4-aligned, G > cs_lo - 16); its bytes before the UDP header are
            // header bytes staged above (cs_lo <= 15 + 14 + 60 < 92)
            fi.head = staged_range_sum(w, G, Lc);
        } else if (kHeadA && (fi.work & 2) && G > Lc) {
            // the checksum bytes before the stream were summed here: a
            // negative head correction (G <= a_end <= 128: all staged)
            fi.head = 0u - staged_range_sum(w, Lc, min(G, fi.g.cs_hi));
        }
        if (kHeadA && (fi.work & 1) && fi.g.de < 0) {
            // events 0 .. -de-1 lie in chunks before the stream: event k's
            // chunk is a0-relative dwords s + 4k .. s + 4k + 3 (s = q / 4, 6..24),
            // aligned here by a 5-step barrel shift (static register indices)
            na = min((uint32_t)(-fi.g.de), a.E);
            const int qd = (16 * (fi.g.c_begin + fi.g.de) + fi.g.q4) >> 2;  // s
            const uint32_t t = (uint32_t)(qd - 6);
            // (a decoded event's dwords end by a0-relative dword 31: j + t <= 24)
            constexpr int NX = 4 * kAEv - 1;
            uint32_t x[NX];
#pragma unroll
            for (int j = 0; j < NX; j++)
                x[j] = j + 6 < 32 ? w[j + 6] : 0u;
#pragma unroll
            for (int b = 4; b >= 0; b--) {
                const bool on = (t >> b) & 1u;
#pragma unroll
                for (int j = 0; j + (1 << b) < NX; j++)
                    x[j] = on ? x[j + (1 << b)] : x[j];
            }
            const uint32_t rr = (uint32_t)fi.g.r;
#pragma unroll
            for (int k = 0; k < kAEv; k++) {
                const uint32_t xx = __builtin_amdgcn_alignbyte(x[4 * k + 1], x[4 * k], rr);      // event bytes 2..5
                const uint32_t yy = __builtin_amdgcn_alignbyte(x[4 * k + 2], x[4 * k + 1], rr);  // event bytes 6..9
                const uint32_t ch = xx & 0xffffu;
                const uint32_t bin = __builtin_amdgcn_perm(yy, xx, 0x0c0c0403u);
                const uint32_t hc = __builtin_amdgcn_ubfe(yy, 16, 3);
                const uint32_t key = __umul24(ch, kHists << 16) + (hc << 16) + bin;
                akey[k] = ch < kChannels && hc < kHists ? key : DQDK_KEY_NONE;  // tristan.c:236-241
            }
        }
    }
#undef FB
}

// udp_audit_checksum's verdict from S = sum of the datagram's LE u16 words
// (check field included as stored): src/tcpip/udp.c:10-20, inet_csum.c:145-216.
__device__ __forceinline__ bool udp_csum_ok(uint32_t S, uint32_t check, uint32_t len16, uint64_t pseudo)
{
    if (len16 >= 7)
        S -= check;                         // udp->check = 0 before summing (udp.c:17)
    uint64_t t = (uint64_t)S + pseudo;      // csum_tcpudp_nofold
    t = (t & 0xffffffffull) + (t >> 32);     // from64to32
    t = (t & 0xffffffffull) + (t >> 32);
    uint32_t f = (uint32_t)t;
    f = (f & 0xffff) + (f >> 16);            // csum_fold
    f = (f & 0xffff) + (f >> 16);
    return ((~f) & 0xffffu) == check;
}

// ---------------------------------------------------------------------------
// Each wave owns 64-frame tiles end to end (no block barriers):
//   phase A  lane l parses frame 64*tile + l (headers staged in VGPRs) and
//            prepares its frame's stream: SRD base/extent, window count,
//            decode shift, checksum head correction;
//   phase B  the wave streams the chunks of its frames as ONE sequence of
//            2-KiB windows (lane = 32 B = two 16-B chunks), kRingW windows
//            in flight across frame boundaries; each frame has its own SRD
//            whose extent ends at the frame's last chunk, so loads past it
//            return zeros (no per-lane bounds tests); per-frame parameters
//            come from the owning lane (readlane), per-frame sums go back to it;
//   phase C  lane l finishes its own frame: checksum verdict, result record
//            (coalesced), KEY_NONE records for non-OK frames.
// Every window issues exactly two loads and two key stores (lanes without an
// event store to an out-of-range offset), so hipcc counts the ring with
// vmcnt(N) on every path instead of draining it.
// ---------------------------------------------------------------------------
#ifndef DQDK_LD_AUX
#define DQDK_LD_AUX 0
#endif
// the fused decode's piece stores: write-back where runs end mid-line (the
// next round completes a partial line in L2), streaming in the lines policy
// (whole lines only: nothing to merge; r05v: 9000 B decode -1.7 %, 1500 B
// +5 % with streaming partial lines)
constexpr int kFstAux = 0, kFstAuxLines = 2;
#ifndef DQDK_ST_AUX
#define DQDK_ST_AUX 0
#endif
constexpr uint32_t kOOB = 0x80000000u;  // buffer offset beyond every SRD's num_records

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
// a VGPR value the compiler cannot see through: per-lane addresses derived
// from it are recomputed where used instead of hoisted out of a loop (live
// across it, they spill)
__device__ __forceinline__ uint32_t opaque(uint32_t v)
{
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// sum over the wave: 4 DPP row shifts, then the four row totals
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    return rdl(x, 15) + rdl(x, 31) + rdl(x, 47) + rdl(x, 63);
}

// inclusive prefix sum over the wave: rows by DPP shifts, then rows 1-3
// take the earlier rows' totals by row broadcasts (no LDS round trips)
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint64_t bytes)
{
    // SRD from readfirstlane'd halves so hipcc can prove it uniform
    // (otherwise every buffer op becomes a waterfall loop: guide T20)
    const uint64_t b = (uint64_t)p;
    const uint64_t ub = (uint64_t)rfl((uint32_t)b) | ((uint64_t)rfl((uint32_t)(b >> 32)) << 32);
    const uint32_t nrec = rfl((uint32_t)(bytes > 0x7fffffffull ? 0x7fffffffull : bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)ub, (short)0, (int)nrec, 0x00020000);
}

// LDS of one rx_decode block: partition bucket counts, per-frame out-of-bounds
// counts and checksum sums (one slot per frame of each wave's tile) and the
// captured last checksum chunk of each frame.  Frame slots are reset by
// their lane in phase C.
constexpr int kLdsOob = 288;                      // [kWaves][64] out-of-bounds events per frame
constexpr int kLdsCnt = kLdsOob + kWaves * 64;
struct DecodeLds {
    uint32_t cnt[kLdsCnt];       // [0, kL1Buckets): keys per L1 bucket (partitioned histogram)
    uint32_t sum[kWaves * 64];   // checksum word sums per frame
    uint32_t sink[64];           // per-lane dump word (frame_sum_add)
    u32x4 tail[kWaves * 64];     // last checksum chunk per frame (tail correction)
    alignas(8) uint32_t fc[kFoldWords];  // folded counters of the block (RxArgs::fold; FoldWord)
};

// Per-frame stream parameters in the owning lane's VGPRs.
//   pk1 = nwin | (de + 8) << 16 | r << 20 | dec << 22 | lw << 23 | th << 24 | tl << 25
//   pk2 = tw | mw << 11 | keep << 22 | sh << 27
// nwin: 2-KiB windows; de: chunk of event 0 (-7..1); r: event shift; dec: decode;
// sh: the first chunk's first dword comes from phase A (fused, parse_frame);
// lw: some window needs per-lane checksum weights (chunks past ct), the
// first such window is mw; tw/tl/th: window/lane/half holding the last
// checksum chunk when it needs a tail correction (tw = 0xffff: none).
struct LaneFrame {
    uint32_t base_lo, base_hi;  // umem + a0 + 16 c_begin + q4
    uint32_t nrec;              // streamed bytes inside the UMEM
    uint32_t pk1, pk2;
    int ct;
};

constexpr uint32_t kNoWin = 0x7ffu;  // (a frame streams at most 513 windows: E <= 65535)

__device__ __forceinline__ uint32_t pk_nwin(uint32_t pk1) { return pk1 & 0xffffu; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const LaneFrame& lf, uint32_t j)
{
    const uint64_t b = (uint64_t)rdl(lf.base_lo, j) | ((uint64_t)rdl(lf.base_hi, j) << 32);
    return __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, (int)rdl(lf.nrec, j), 0x00020000);
}

// Wave-uniform view of the frame being processed.
struct PFrame {
    uint32_t nwin, de, r, Ef, lw, th, tl, tw, mw;  // Ef = events to decode (0: frame not decoded)
    int ct;
    uint32_t keep;  // checksum bytes in the last checksum chunk (tail correction when < 16)
    uint32_t sh, hw;  // fused first-line hand-off: lane 0's first chunk starts with hw
};

__device__ __forceinline__ void pframe(const RxArgs& a, const LaneFrame& lf, uint32_t j, PFrame& P)
{
    const uint32_t pk1 = rdl(lf.pk1, j), pk2 = rdl(lf.pk2, j);
    P.nwin = pk1 & 0xffffu;
    P.de = ((pk1 >> 16) & 15u) - 8u;  // (u32: e = j - de wraps to j + events phase A took)
    P.r = (pk1 >> 20) & 3u;
    P.Ef = (pk1 & (1u << 22)) ? a.E : 0u;
    P.lw = (pk1 >> 23) & 1u;
    P.th = (pk1 >> 24) & 1u;
    P.tl = pk1 >> 25;
    P.tw = pk2 & kNoWin;
    P.mw = (pk2 >> 11) & kNoWin;
    P.keep = (pk2 >> 22) & 31u;
    P.sh = (pk2 >> 27) & 1u;
    P.hw = P.sh ? rdl((uint32_t)lf.ct, j) : 0u;
    P.ct = P.lw ? (int)rdl((uint32_t)lf.ct, j) : 0;
}

__device__ __forceinline__ void lds_add_u32(uint32_t lds_addr, uint32_t v)
{
    asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr), "v"(v) : "memory");
}

// The frame's checksum word sum into its LDS slot.  One add from every lane
// to one address serialises 64 LDS cycles (PMC: bank-conflict cycles were
// 83 % of the fused decode's LDS cycles); instead the row sums are formed by
// DPP and only the four row-end lanes add to the slot, the others to their
// own sink word (distinct banks).
#ifndef DQDK_SUM_DPP
#define DQDK_SUM_DPP 1
#endif
__device__ __forceinline__ void frame_sum_add(uint32_t* slot, uint32_t* sink, uint32_t t, bool row_end)
{
#if DQDK_SUM_DPP
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x111, 0xf, 0xf, false);  // row_shr:1
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x112, 0xf, 0xf, false);  // row_shr:2
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x114, 0xf, 0xf, false);  // row_shr:4
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x118, 0xf, 0xf, false);  // row_shr:8
    lds_add_u32((uint32_t)(uintptr_t)(row_end ? slot : sink), t);
#else
    (void)sink;
    (void)row_end;
    lds_add_u32((uint32_t)(uintptr_t)slot, t);
#endif
}

// One event per 16-B chunk v (event byte 2 at byte r of v.x): key record
// store, then one LDS count: the key's L1 bucket, the frame's OOB slot for
// an out-of-bounds event (lanes without an event do no LDS count).
__device__ __forceinline__ void decode_chunk(const u32x4& v, uint32_t r, uint32_t e, uint32_t Ef, uint32_t kbase,
                                             uint32_t oob_slot, __amdgpu_buffer_rsrc_t keys_rsrc, uint32_t* cnt)
{
    const uint32_t x = __builtin_amdgcn_alignbyte(v.y, v.x, r);  // event bytes 2..5
    const uint32_t y = __builtin_amdgcn_alignbyte(v.z, v.y, r);  // event bytes 6..9
    const uint32_t ch = x & 0xffffu;
    const uint32_t bin = __builtin_amdgcn_perm(y, x, 0x0c0c0403u);   // event bytes 5,6 = energy >> 8
    const uint32_t hc = __builtin_amdgcn_ubfe(y, 16, 3);             // hist_class:3
    uint32_t key = __umul24(ch, kHists << 16) + (hc << 16) + bin;  // ((ch*6 + hc) << 16) | bin
    key = ch < kChannels ? key : DQDK_KEY_NONE;
    key = hc < kHists ? key : DQDK_KEY_NONE;
    const bool has = e < Ef;
    __builtin_amdgcn_raw_buffer_store_b32(key, keys_rsrc, has ? kbase + 4u * e : kOOB, 0, DQDK_ST_AUX);
    // KEY_NONE >> kL1Shift = 2047 > oob_slot > every bucket
    // lanes without an event stay out of the LDS: at 1500 B 37 of a window's
    // 128 chunk slots carry none, and one shared sink word serialised them
    if (has)
        atomicAdd(&cnt[min(key >> kL1Shift, oob_slot)], 1u);
}

// T = sum of the LE 16-bit words at even addresses of a chunk (chunk starts
// are 4-aligned, so a dword's two halves)
__device__ __forceinline__ uint32_t csum_chunk(const u32x4& v, u16x2 wt, uint32_t acc)
{
    acc = __builtin_amdgcn_udot2(as_u16x2(v.x), wt, acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(v.y), wt, acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(v.z), wt, acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(v.w), wt, acc, false);
    return acc;
}

// both chunks of a lane interleaved: two independent dot2 chains
__device__ __forceinline__ void csum_pair(const u32x4& v0, const u32x4& v1, u16x2 w0, u16x2 w1, uint32_t& acc0,
                                          uint32_t& acc1)
{
    acc0 = __builtin_amdgcn_udot2(as_u16x2(v0.x), w0, acc0, false);
    acc1 = __builtin_amdgcn_udot2(as_u16x2(v1.x), w1, acc1, false);
    acc0 = __builtin_amdgcn_udot2(as_u16x2(v0.y), w0, acc0, false);
    acc1 = __builtin_amdgcn_udot2(as_u16x2(v1.y), w1, acc1, false);
    acc0 = __builtin_amdgcn_udot2(as_u16x2(v0.z), w0, acc0, false);
    acc1 = __builtin_amdgcn_udot2(as_u16x2(v1.z), w1, acc1, false);
    acc0 = __builtin_amdgcn_udot2(as_u16x2(v0.w), w0, acc0, false);
    acc1 = __builtin_amdgcn_udot2(as_u16x2(v1.w), w1, acc1, false);
}

// Window wp of frame P (owned by lane `slot`): lane l holds chunks
// 128 wp + l (v0) and 128 wp + 64 + l (v1), so each load, store and sum is
// one contiguous 1-KiB span.  Chunks past the frame's extent read zeros.
__device__ __forceinline__ void process_window(const RxArgs& a, const PFrame& P, uint32_t slot, uint32_t wslot0,
                                               uint32_t wp, const u32x4& v0, const u32x4& v1, int lane, bool active,
                                               __amdgpu_buffer_rsrc_t keys_rsrc, uint32_t& acc0, uint32_t& acc1,
                                               DecodeLds& lds)
{
    const uint32_t jw = (uint32_t)kWinChunks * wp;
    if (active && wp >= P.mw) {
        // rare: E*16 reaches past the datagram, chunks past ct carry no checksum bytes
        const int j0 = (int)jw + lane;
        csum_pair(v0, v1, j0 <= P.ct ? u16x2{1, 1} : u16x2{0, 0}, j0 + 64 <= P.ct ? u16x2{1, 1} : u16x2{0, 0}, acc0,
                  acc1);
    } else {
        // (inactive windows read zeros; sums of frames without a checksum are ignored)
        csum_pair(v0, v1, u16x2{1, 1}, u16x2{1, 1}, acc0, acc1);
    }
    if (active && wp == P.tw) {  // the last checksum chunk, for phase C's tail correction
        if (lane == (int)P.tl)
            lds.tail[wslot0 + slot] = P.th ? v1 : v0;
    }
    // records of this wave tile live at keys_rsrc + (slot*E + e)*4
    const uint32_t Ef = active ? P.Ef : 0u;
    const uint32_t e0 = jw + (uint32_t)lane - P.de;
    const uint32_t kbase = slot * a.E * 4u;
    const uint32_t oob_slot = (uint32_t)kLdsOob + wslot0 + slot;
    decode_chunk(v0, P.r, e0, Ef, kbase, oob_slot, keys_rsrc, lds.cnt);
    decode_chunk(v1, P.r, e0 + 64u, Ef, kbase, oob_slot, keys_rsrc, lds.cnt);
}

// ---- phase A: lane parses frame i and prepares its stream (shared by both decodes) ----
template <bool kHeadA = false, bool kHalf = false>
__device__ __forceinline__ void phase_a(const RxArgs& a, uint32_t i, bool live, FrameInfo& fi,
                                        dqdk_gpu_rx_result_t& r, LaneFrame& lf, bool& stream,
                                        uint32_t (&akey)[kAEv], uint32_t& na, uint32_t& hw)
{
    bool needB = false, sh = false;
    na = 0;
    hw = 0;
#pragma unroll
    for (int k = 0; k < kAEv; k++)
        akey[k] = DQDK_KEY_NONE;
    if (live)
        parse_frame<kHeadA, kHalf>(a, i, fi, r, needB, akey, na, hw, sh);
    stream = false;
    lf.base_lo = lf.base_hi = lf.nrec = lf.pk1 = 0;
    lf.pk2 = kNoWin | (kNoWin << 11);
    lf.ct = -1;
    if (needB) {
        const Geo& g = fi.g;
        stream = g.nwin > 0;  // (no stream: an empty datagram, or all of it in phase A; phase C checks it)
        const uint64_t boff = (fi.addr & ~15ull) + 16ull * (uint64_t)g.c_begin + (uint64_t)g.q4;
        const uint64_t base = (uint64_t)a.umem + boff;
        const uint64_t ext = 16ull * (uint64_t)g.nch;
        const uint64_t room = a.umem_size > boff ? a.umem_size - boff : 0ull;
        lf.base_lo = (uint32_t)base;
        lf.base_hi = (uint32_t)(base >> 32);
        lf.nrec = (uint32_t)(ext < room ? ext : room);
        const bool cs = fi.work & 2;
        const bool lw = cs && g.ct < g.nch - 1;   // chunks past ct are streamed (decode reaches further)
        const bool tc = cs && g.ct >= 0 && g.keep < 16;
        const uint32_t ct = (uint32_t)(g.ct < 0 ? 0 : g.ct);
        lf.pk1 = ((uint32_t)g.nwin & 0xffffu) | (((uint32_t)(g.de + 8) & 15u) << 16) | (((uint32_t)g.r & 3u) << 20) |
                 ((fi.work & 1u) << 22) | ((lw ? 1u : 0u) << 23) | (((ct >> 6) & 1u) << 24) | ((ct & 63u) << 25);
        const uint32_t tw = tc ? ct / (uint32_t)kWinChunks : kNoWin;
        const uint32_t mw = lw ? (uint32_t)(g.ct + 1) / (uint32_t)kWinChunks : kNoWin;
        lf.pk2 = tw | (mw << 11) | (((uint32_t)g.keep & 31u) << 22) | ((sh && stream ? 1u : 0u) << 27);
        lf.ct = sh ? (int)hw : g.ct;  // (sh frames never need ct: see parse_frame)
    }
    if (!stream)
        lf.pk1 = 0;
}

// Word sum of the bytes [keep, 16) of a frame's last checksum chunk: the
// part of it past the datagram (the odd-length over-read byte is inside
// keep), which the streamed sum must not contain.
__device__ __forceinline__ uint32_t tail_corr(const u32x4& tail, int keep)
{
    const uint32_t tw4[4] = {tail.x, tail.y, tail.z, tail.w};
    uint32_t corr = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int lo = keep - 4 * d;  // bytes of dword d inside the datagram
        const uint32_t m = lo <= 0 ? 0xffffffffu : lo >= 4 ? 0u : (0xffffffffu << (8 * lo));
        corr = __builtin_amdgcn_udot2(as_u16x2(tw4[d] & m), u16x2{1, 1}, corr, false);
    }
    return corr;
}

// ---- phase C: lane finishes its own frame (checksum verdict, result) ----
__device__ __forceinline__ void phase_c(const RxArgs& a, uint32_t i, bool live, bool stream, const FrameInfo& fi,
                                        dqdk_gpu_rx_result_t& r, uint32_t sum_t, uint32_t sum_oob, const u32x4& tail)
{
    if (live) {
        if (fi.work & 2) {
            // tail correction: bytes [keep, 16) of the last checksum chunk lie
            // past the datagram (the odd-length over-read byte is inside keep)
            // (the fused decode subtracted it in the window loop: tail is 0 there)
            // (no stream: sum_t is 0 and the head correction carries phase A's
            // sum, or nothing for an empty datagram)
            const uint32_t corr = stream && fi.g.ct >= 0 && fi.g.keep < 16 ? tail_corr(tail, fi.g.keep) : 0u;
            // udp_csum sums LE words from the UDP start.  tsum summed the words
            // at even addresses: the same words when the UDP header starts at an
            // even address; otherwise every word is byte-swapped, and the one's
            // complement sum of swapped words is the swapped sum (the value
            // mod 0xffff is all udp_csum_ok depends on; + 0xffff keeps the
            // check subtraction from wrapping)
            const uint32_t tsum = sum_t - fi.head - corr;
            const bool even = !fi.odd;
            uint32_t f = (tsum & 0xffffu) + (tsum >> 16);
            f = (f & 0xffffu) + (f >> 16);
            const uint32_t S = even ? tsum : (((f >> 8) | (f << 8)) & 0xffffu) + 0xffffu;
            if (!udp_csum_ok(S, fi.check, fi.len16, fi.pseudo))
                r.status = DQDK_RX_INVALID_UDP_CSUM;
        }
        // histogram_event's rejections: none without a histogram (E <= 65535, so no clamp);
        // sum_oob is 0 for a frame nothing was decoded from
        r.oob_events = (uint16_t)(r.status == DQDK_RX_OK && a.histo ? sum_oob : 0u);
    }
    if (live) {
        if (r.status != DQDK_RX_OK && r.status != DQDK_RX_EMPTY) {
            r.datalen = 0;
            r.payload_off = 0;
        }
        a.res[i] = r;
        if ((fi.work & 2) && (a.flags & DQDK_GPU_F_CSUM_WRITEBACK)) {  // udp.c:17 side effect
            const uint64_t ck = a.desc[i].addr + 14 + fi.hs + 6;
            if (ck + 2 <= a.umem_size) {
                uint8_t* p = const_cast<uint8_t*>(a.umem) + ck;
                p[0] = 0;
                p[1] = 0;
            }
        }
    }
}

// Folded counters (RxArgs::fold): the block's sums of rx_count's per-frame
// accounting (src/dqdk.c:252-322 per-packet form), in LDS then blk_cnt.
enum FoldWord { F_FILT, F_FRAMES, F_IP, F_UDP, F_EMPTY, F_OK, F_BYTES_LO, F_BYTES_HI, F_OOB, F_FAIL, F_NWORDS };

// One wave's frames of a super-tile into the block's folded counters
// (ballots and DPP sums; lane 0 adds to LDS).  i: the lane's frame index.
__device__ __forceinline__ void fold_frames(const RxArgs& a, uint32_t* fc, bool live, const dqdk_gpu_rx_result_t& r,
                                            uint32_t i, int lane)
{
    const uint32_t st = r.status;
    const bool inb = st != DQDK_RX_FILTER_DROP && st != DQDK_RX_FILTER_PASS;
    const bool ok = live && st == DQDK_RX_OK;
    const bool fail = live && inb && st != DQDK_RX_OK;
    const uint64_t mfail = __ballot(fail);
    uint32_t ifail = fail ? i : ~0u;  // the wave's first failing frame
    if (mfail) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            ifail = min(ifail, (uint32_t)__shfl_xor((int)ifail, o));
    }
    const uint32_t filt = (uint32_t)__builtin_popcountll(__ballot(live && !inb));
    const uint32_t frames = (uint32_t)__builtin_popcountll(__ballot(live && inb));
    const uint32_t ip = (uint32_t)__builtin_popcountll(
        __ballot(live && (st == DQDK_RX_INVALID_IP || st == DQDK_RX_INVALID_IP_CSUM)));
    const uint32_t udp = (uint32_t)__builtin_popcountll(
        __ballot(live && (st == DQDK_RX_INVALID_UDP || st == DQDK_RX_INVALID_UDP_CSUM)));
    const uint32_t empty = (uint32_t)__builtin_popcountll(__ballot(live && st == DQDK_RX_EMPTY));
    const uint32_t nok = (uint32_t)__builtin_popcountll(__ballot(ok));
    // datalen is a u32 that wraps to ~4 G for udplen < 8 (dqdk.c:205): the
    // wave sums its 16-bit halves (64 x 65535 < 2^32 each)
    const uint32_t dl = ok ? r.datalen : 0u;
    const uint64_t bytes = (uint64_t)wave_sum_dpp(dl & 0xffffu) + ((uint64_t)wave_sum_dpp(dl >> 16) << 16);
    const uint32_t oob = wave_sum_dpp(ok && a.histo ? (uint32_t)r.oob_events : 0u);
    if (lane == 0) {
        if (filt)
            atomicAdd(&fc[F_FILT], filt);
        if (frames)
            atomicAdd(&fc[F_FRAMES], frames);
        if (ip)
            atomicAdd(&fc[F_IP], ip);
        if (udp)
            atomicAdd(&fc[F_UDP], udp);
        if (empty)
            atomicAdd(&fc[F_EMPTY], empty);
        if (nok)
            atomicAdd(&fc[F_OK], nok);
        if (bytes)
            atomicAdd((unsigned long long*)&fc[F_BYTES_LO], (unsigned long long)bytes);  // (u64 per block)
        if (oob)
            atomicAdd(&fc[F_OOB], oob);
        if (mfail)
            atomicMin(&fc[F_FAIL], ifail);
    }
}

// The block's folded counters into the batch's accumulators (a.blk_cnt as
// u64 words: device atomics, which execute at the memory side, so no fence
// and no L2 write-back -- an agent-scope fence here wrote back every XCD's
// dirty piece lines under the still-running blocks: decode +0.1 ms); the
// last block (ticket, taken once its own adds have returned) swaps the
// totals out, resetting them, and publishes the batch: batch_scratch [0] =
// first failing frame (n: none), [1..12] = dqdk_gpu_counters_t of the batch,
// each added to cum -- what rx_abort + rx_count write for a per-packet batch.
__device__ __forceinline__ void fold_publish(const RxArgs& a, uint32_t* fc, int tid)
{
    __shared__ uint32_t last;
    __shared__ uint64_t tot[F_NWORDS];
    unsigned long long* acc = (unsigned long long*)a.blk_cnt;  // [F_NWORDS] (F_BYTES_HI unused)
    __syncthreads();  // every wave's fold_frames adds are in LDS
    if (tid < 64) {
        uint64_t r = 0;
        if (tid < F_NWORDS && tid != F_BYTES_HI) {
            const uint64_t v = tid == F_BYTES_LO ? *(const uint64_t*)&fc[F_BYTES_LO] : (uint64_t)fc[tid];
            r = tid == F_FAIL ? atomicMin(&acc[F_FAIL], (unsigned long long)v) : atomicAdd(&acc[tid], (unsigned long long)v);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(r) : "memory");  // the adds are performed before the ticket
        if (tid == 0)
            last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last)
        return;  // (block-uniform)
    if (tid < F_NWORDS && tid != F_BYTES_HI)
        tot[tid] = atomicExch(&acc[tid], tid == F_FAIL ? ~0ull : 0ull);  // the totals; reset for the next batch
    __syncthreads();
    if (tid == 0) {
        const uint64_t n = a.n;
        const uint64_t fail = tot[F_FAIL] < n ? tot[F_FAIL] : n;
        const uint64_t c[12] = {tot[F_FRAMES], tot[F_FRAMES], tot[F_BYTES_LO], tot[F_IP],
                                tot[F_UDP],    fail < n ? 1ull : 0ull, tot[F_OK] * a.E, tot[F_BYTES_LO],
                                tot[F_OOB],    tot[F_EMPTY], tot[F_FILT], fail};
        unsigned long long* cum = (unsigned long long*)a.cum;
        a.batch_scratch[0] = fail;
#pragma unroll
        for (int k = 0; k < 12; k++) {
            a.batch_scratch[1 + k] = c[k];
            if (k < 11 && c[k])
                atomicAdd(&cum[k], (unsigned long long)c[k]);
        }
        cum[11] = fail;  // first_abort_idx of this batch
#pragma unroll
        for (int k = 1 + 12; k < 17; k++)  // (the rest of the per-batch words the unfolded decode resets)
            a.batch_scratch[k] = 0;
        *a.ticket = 0;
    }
}

__device__ __forceinline__ void decode_wave_tile(const RxArgs& a, uint32_t tile, uint32_t F, int lane,
                                                 uint32_t wave, DecodeLds& lds)
{
    const uint32_t i = tile * F + lane;
    const bool live = (uint32_t)lane < F && i < a.n;
    const uint32_t wslot0 = wave * 64;

    // ---- phase A: lane parses frame i ----
    FrameInfo fi;
    dqdk_gpu_rx_result_t r;
    LaneFrame lf;
    bool stream;
    uint32_t akey[kAEv], na, hw;
    phase_a<false, true>(a, i, live, fi, r, lf, stream, akey, na, hw);

    // ---- phase B: stream the frames ----
    const uint64_t smask0 = __ballot(stream);
    if (smask0) {
        const int total = (int)wave_sum_dpp(pk_nwin(lf.pk1));
        const __amdgpu_buffer_rsrc_t keys_rsrc =
            uniform_rsrc(a.keys + (uint64_t)tile * F * a.E, a.keys ? (uint64_t)F * a.E * 4u : 0u);
        const uint32_t lane16 = (uint32_t)lane * 16u;
        // load cursor
        uint64_t lmask = smask0;
        uint32_t jl = (uint32_t)__builtin_ctzll(lmask);
        uint32_t wl = 0, lnwin = pk_nwin(rdl(lf.pk1, jl));
        __amdgpu_buffer_rsrc_t lrs = frame_rsrc(lf, jl);
        auto issue = [&](u32x4& d0, u32x4& d1) {
            const uint32_t vo = lane16 + (lmask != 0 ? wl * kWinBytes : kOOB);
            d0 = __builtin_amdgcn_raw_buffer_load_b128(lrs, vo, 0, DQDK_LD_AUX);
            d1 = __builtin_amdgcn_raw_buffer_load_b128(lrs, vo + 1024u, 0, DQDK_LD_AUX);
            if (lmask != 0 && ++wl == lnwin) {
                wl = 0;
                lmask &= lmask - 1;
                if (lmask) {
                    jl = (uint32_t)__builtin_ctzll(lmask);
                    lnwin = pk_nwin(rdl(lf.pk1, jl));
                    lrs = frame_rsrc(lf, jl);
                }
            }
        };
        u32x4 b0[kRingW], b1[kRingW];
#pragma unroll
        for (int d = 0; d < kRingW; d++) {
            // two dropped stores per window, as in the loop body (store, store,
            // load, load): the loop is entered with the same vmcnt pattern it
            // repeats, so the wait for window d is vmcnt(4 * (kRingW - 1)), not
            // the prologue's shorter count (distinct offsets: not merged)
            __builtin_amdgcn_raw_buffer_store_b32(0u, keys_rsrc, kOOB + lane16 + 8u * d, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(0u, keys_rsrc, kOOB + lane16 + 8u * d + 4u, 0, 0);
            issue(b0[d], b1[d]);
        }
        // process cursor
        uint64_t pmask = smask0;
        uint32_t jp = (uint32_t)__builtin_ctzll(pmask);
        uint32_t wp = 0;
        PFrame P;
        pframe(a, lf, jp, P);
        uint32_t acc0 = 0, acc1 = 0;
        for (int k = 0; k < total; k += kRingW) {
#pragma unroll
            for (int d = 0; d < kRingW; d++) {
                const bool active = k + d < total;
                process_window(a, P, jp, wslot0, wp, b0[d], b1[d], lane, active, keys_rsrc, acc0, acc1, lds);
                if (active && ++wp == P.nwin) {
                    // the frame's checksum word sum to its LDS slot: every lane adds into
                    // one address (inline asm: the compiler's atomic optimizer would turn
                    // a uniform-address atomicAdd into a 64-step readlane loop)
                    frame_sum_add(&lds.sum[wslot0 + jp], &lds.sink[lane], acc0 + acc1, (lane & 15) == 15);
                    acc0 = acc1 = 0;
                    wp = 0;
                    pmask &= pmask - 1;
                    if (pmask) {
                        jp = (uint32_t)__builtin_ctzll(pmask);
                        pframe(a, lf, jp, P);
                    }
                }
                issue(b0[d], b1[d]);
            }
        }
    }

    // ---- phase C: lane finishes its own frame ----
    const uint32_t my = wslot0 + (uint32_t)lane;
    const uint32_t sum_t = lds.sum[my], sum_oob = lds.cnt[kLdsOob + my];
    lds.sum[my] = 0;
    lds.cnt[kLdsOob + my] = 0;
    phase_c(a, i, live, stream, fi, r, sum_t, sum_oob, lds.tail[my]);
    if (a.fold)  // per-packet counters summed here: no rx_abort / rx_count launches
        fold_frames(a, lds.fc, live, r, i, lane);
    // the partitioned histogram reads records by index only: every non-OK
    // frame gets KEY_NONE records (rare; after this wave's speculative stores)
    const bool fill = live && a.cnt1 && a.keys && a.E && r.status != DQDK_RX_OK;
    if (__ballot(fill)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (fill) {
            uint32_t* k = a.keys + (uint64_t)i * a.E;
            for (uint32_t e = 0; e < a.E; e++)
                k[e] = DQDK_KEY_NONE;
        }
    }
}

__device__ __forceinline__ void decode_block(const RxArgs& a, DecodeLds& lds)
{
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wave = rfl((uint32_t)(tid >> 6));
    for (int b = tid; b < kLdsCnt; b += kTile)
        lds.cnt[b] = 0;
    lds.sum[tid] = 0;
    if (tid < kFoldWords)
        lds.fc[tid] = tid == F_FAIL ? ~0u : 0u;
    __syncthreads();
    // per-batch state reset (folded counters: the last block's fold_publish
    // writes these words instead)
    if (!a.fold && blockIdx.x == 0 && tid < 17)
        a.batch_scratch[tid] = tid == 0 ? (uint64_t)a.n : 0ull;

    const uint32_t F = a.tile_frames ? a.tile_frames : 64u;
    const uint32_t ntiles = (a.n + F - 1) / F;
    for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += gridDim.x * kWaves)
        decode_wave_tile(a, t, F, lane, wave, lds);

    if (a.cnt1) {
        __syncthreads();
        for (int b = tid; b < kL1Buckets; b += kTile)
            if (lds.cnt[b])
                atomicAdd(&a.cnt1[b], lds.cnt[b]);
    }
    if (a.fold)
        fold_publish(a, lds.fc, tid);
}

__global__ void __launch_bounds__(kTile) rx_decode_kernel(RxArgs a)
{
    __shared__ DecodeLds lds;
    decode_block(a, lds);
}

// ===========================================================================
// Frame-processor plugin: payloads staged by dqdk_gpu_frame_processor, one
// per tristan_process(payload, datalen, 1) call (src/tristan.c:308-330).  A
// wave takes one payload at a time: lane e decodes events e, e + 64, ...
// (16-B aligned loads: the staging stride is E * 16) into frame-order
// records, exactly histogram_event's key and bounds (src/tristan.c:233-245);
// lane 0 writes the call's result record (datalen, rejected events) for
// rx_count.  The records feed the records-path histogram (atomic or
// partitioned), as rx_decode's do.
// ===========================================================================
__global__ void __launch_bounds__(kTile) fp_decode_kernel(PayloadArgs a)
{
    __shared__ uint32_t cnt[kL1Buckets];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    if (a.cnt1) {
        for (int b = tid; b < kL1Buckets; b += kTile)
            cnt[b] = 0;
        __syncthreads();
    }
    if (blockIdx.x == 0 && tid < 17)
        a.batch_scratch[tid] = tid == 0 ? (uint64_t)a.n : 0ull;  // per-batch state reset
    const uint32_t gw = (blockIdx.x * kTile + (uint32_t)tid) >> 6;
    const uint32_t nw = (gridDim.x * kTile) >> 6;
    for (uint32_t p = gw; p < a.n; p += nw) {
        uint32_t oob = 0;
        if (a.histo) {
            const u32x4* ev = (const u32x4*)(a.stage + (uint64_t)p * a.E * 16u);
            uint32_t* k = a.keys + (uint64_t)p * a.E;
            for (uint32_t e = (uint32_t)lane; e < a.E; e += 64) {
                const u32x4 v = __builtin_nontemporal_load(&ev[e]);
                const uint32_t ch = v.x >> 16;             // event bytes 2..3
                const uint32_t bin = (v.y >> 8) & 0xffffu;  // event bytes 5,6 = energy >> 8
                const uint32_t hc = v.z & 7u;               // byte 8, hist_class:3
                const bool inb = ch < kChannels && hc < kHists;
                const uint32_t key = __umul24(ch, kHists << 16) + (hc << 16) + bin;
                k[e] = inb ? key : DQDK_KEY_NONE;
                oob += inb ? 0u : 1u;
                if (inb && a.cnt1)
                    atomicAdd(&cnt[key >> kL1Shift], 1u);
            }
            oob = wave_sum_dpp(oob);
        }
        if (lane == 0) {
            dqdk_gpu_rx_result_t r;
            r.datalen = a.len[p];
            r.status = DQDK_RX_OK;  // process_frame calls the processor only for datalen != 0
            r.payload_off = 0;
            r.oob_events = (uint16_t)oob;  // E <= 65535
            a.res[p] = r;
        }
    }
    if (a.cnt1) {
        __syncthreads();
        for (int b = tid; b < kL1Buckets; b += kTile)
            if (cnt[b])
                atomicAdd(&a.cnt1[b], cnt[b]);
    }
}

// ===========================================================================
// Fused decode: rx_decode + rx_part1 in one persistent kernel.  A block of
// kFWaves waves takes kFWaves 64-frame tiles at a time (a super-tile); its
// waves stream their frames exactly as rx_decode does, but a decoded key goes
// to the block's LDS stage of its L1 bucket (a returning LDS atomic gives its
// slot) instead of to a frame-order record.  Every round_windows windows the
// block synchronises and every bucket's staged run is appended to the block's
// piece of that bucket (fused_geom's [bucket][block][cap] region): the
// piece cursors are private to the block (one per lane of the owning wave,
// in a VGPR), so no device atomic is on the path.  Keys past kFCap in a round,
// or past a full piece, go to the block's private overflow region and from
// there to the overflow list, which rx_part1 groups like frame-order records.
// Frames decoded but later failing the UDP checksum are listed for rx_fixup.
// ===========================================================================
// The stage holds each bucket's keys as its piece will, three 21-bit
// bucket-local keys to an 8-B word in slot order (k0 | k1 << 21 | k2 << 42):
// a key is OR-ed into its field (the word is zero until then: a flushed word
// is zeroed), and a flush copies whole words, unchanged, to the piece.
constexpr uint32_t kStageWords = kL1Buckets * kFCapW;
struct FusedLds {
    alignas(16) uint64_t stage[kStageWords + 64];  // (+64: the flush reads up to 128 words a bucket; the OR sinks)
    uint32_t csink[64];              // the lanes' count sinks (no event)
    uint32_t scnt[kL1Buckets + 4];   // staged keys per bucket this round (returning LDS atomics)
    uint32_t sum[kFWaves * 64];      // checksum word sums per frame
    uint32_t oob[kFWaves * 64];      // out-of-bounds events per frame
    uint32_t wtot[kFWaves];          // windows of each wave's tile
    uint32_t ovf_n;                  // keys in this block's private overflow region
    alignas(8) uint32_t fc[kFoldWords];  // folded counters of the block (FoldWord; the bytes word pair is a u64)
};

// A frame the fused decode staged but whose final status is not OK (it
// failed the UDP checksum): its events are subtracted from the table's base
// plane (u32 wrap: +1 later, -1 now, leaves every bin exact), the wave's
// lanes taking its events in turn.  Event bytes are read as the decode read
// them (zeros at or past umem_size).  (Before round 6 the frame was listed
// and rx_part1 took it back, a launch per batch.)
__device__ __forceinline__ void takeback_frame(const RxArgs& a, uint32_t i, uint32_t lane)
{
    const uint64_t addr = a.desc[i].addr;
    const uint64_t ihl_at = addr + 14;
    const uint32_t ihl = ihl_at < a.umem_size ? (a.umem[ihl_at] & 0xfu) : 0u;
    const uint64_t p = addr + 14 + 4 * ihl + 8;  // get_udp_payload's payload (dqdk.c:205-206)
    for (uint32_t e = lane; e < a.E; e += 64) {
        uint8_t ev[10];
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const uint64_t o = p + 16ull * e + (uint64_t)j;
            ev[j] = o < a.umem_size ? a.umem[o] : (uint8_t)0;
        }
        const uint32_t ch = ev[2] | ((uint32_t)ev[3] << 8);
        const uint32_t hc = ev[8] & 7u;
        const uint32_t bin = ev[5] | ((uint32_t)ev[6] << 8);
        if (ch < kChannels && hc < kHists)
            __hip_atomic_fetch_sub(&a.hist[(ch * kHists + hc) * DQDK_TRISTAN_BINS + bin], 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Block barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release + acquire: on gfx950 that is s_waitcnt vmcnt(0) before s_barrier,
// which would wait for every ring load in flight and every run store of the
// flush at each round.  The rounds only exchange LDS data, for which
// lgkmcnt(0) (this wave's LDS operations performed) is enough.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A key for the block's private overflow region at `slot` (valid lanes only):
// the region holds ovf_blk_cap keys; past that (a pathological spectrum) the
// key goes straight to the table's base plane by a relaxed device atomic --
// the reference's ++ (src/tristan.c:243); exact, since a bin's value is base
// + low (mod 2^32).  The store is issued by every lane (dropped at kOOB), the
// atomic only in this rare branch.
__device__ __forceinline__ void ovf_put(const RxArgs& a, __amdgpu_buffer_rsrc_t ovf_rsrc, uint32_t key, bool valid,
                                        uint32_t slot)
{
    const bool fits = valid && slot < a.ovf_blk_cap;
    __builtin_amdgcn_raw_buffer_store_b32(key, ovf_rsrc, fits ? 4u * slot : kOOB, 0, 0);
    if (valid && !fits)
        __hip_atomic_fetch_add(&a.hist[key], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A staged key into its field: slot s of bucket b is field s % 3 of word
// s / 3 (s < kFCap); a lane without one ORs 0 into its sink word.
__device__ __forceinline__ void stage_key(FusedLds& lds, bool st, uint32_t b, uint32_t s, uint32_t key, uint32_t lane)
{
    const uint32_t q = __umulhi(s, 0xaaaaaaabu) >> 1, f = s - 3u * q;
    uint64_t* const wd = st ? &lds.stage[b * (uint32_t)kFCapW + q] : &lds.stage[kStageWords + (lane & 31u)];
    const uint64_t v = st ? (uint64_t)(key & kTripleMask) << (kL1Shift * f) : 0ull;
    __hip_atomic_fetch_or(wd, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Both chunks of a window at once, without divergent branches: every lane
// issues two returning LDS adds (an event's bucket stage count, a frame's
// out-of-bounds count, or -- lanes without an event -- a private sink word of
// the lane), one wait, then two stage stores (a slot past kFCap, or no event:
// the lane's sink word).  The stage counts' latency is paid once per window
// instead of once per chunk, and no exec mask is saved or restored.  Keys
// past kFCap (rare) go to the block's overflow region behind one
// wave-uniform branch.
__device__ __forceinline__ void fused_pair(const RxArgs& a, const u32x4& va, const u32x4& vb, uint32_t r, uint32_t e0,
                                           uint32_t Ef, uint32_t oob_slot, FusedLds& lds,
                                           __amdgpu_buffer_rsrc_t ovf_rsrc, uint32_t lane)
{
    uint32_t key[2], b[2];
    uint32_t* cnt[2];
    bool ink[2];
    uint32_t* const sink = &lds.csink[lane];  // (the lane's count sink)
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const u32x4& v = c ? vb : va;
        const uint32_t x = __builtin_amdgcn_alignbyte(v.y, v.x, r);  // event bytes 2..5
        const uint32_t y = __builtin_amdgcn_alignbyte(v.z, v.y, r);  // event bytes 6..9
        const uint32_t ch = x & 0xffffu;
        const uint32_t bin = __builtin_amdgcn_perm(y, x, 0x0c0c0403u);  // event bytes 5,6 = energy >> 8
        const uint32_t hc = __builtin_amdgcn_ubfe(y, 16, 3);            // hist_class:3
        key[c] = __umul24(ch, kHists << 16) + (hc << 16) + bin;        // ((ch*6 + hc) << 16) | bin
        const bool inb = ch < kChannels && hc < kHists;                 // tristan.c:236-241
        const bool has = e0 + 64u * c < Ef;
        b[c] = min(key[c] >> kL1Shift, (uint32_t)kL1Buckets - 1);
        ink[c] = has && inb;
        cnt[c] = has ? (inb ? &lds.scnt[b[c]] : &lds.oob[oob_slot]) : sink;
    }
    const uint32_t s0 = atomicAdd(cnt[0], 1u);
    const uint32_t s1 = atomicAdd(cnt[1], 1u);
    const bool st0 = ink[0] && s0 < (uint32_t)kFCap, st1 = ink[1] && s1 < (uint32_t)kFCap;
    stage_key(lds, st0, b[0], s0, key[0], lane);
    stage_key(lds, st1, b[1], s1, key[1], lane);
    const bool ov0 = ink[0] && s0 >= (uint32_t)kFCap, ov1 = ink[1] && s1 >= (uint32_t)kFCap;
    const uint64_t m0 = __ballot(ov0), m1 = __ballot(ov1);
    if (m0 | m1) {  // rare: overflow slots, one LDS atomic per wave
        const uint32_t n0 = (uint32_t)__builtin_popcountll(m0);
        const uint32_t first = (uint32_t)__builtin_ctzll(m0 | m1);
        uint32_t base = 0;
        if (lane == first)
            base = atomicAdd(&lds.ovf_n, n0 + (uint32_t)__builtin_popcountll(m1));
        base = rdl(base, first);
        const uint32_t r0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
        const uint32_t r1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
        ovf_put(a, ovf_rsrc, key[0], ov0, base + r0);
        ovf_put(a, ovf_rsrc, key[1], ov1, base + n0 + r1);
    }
}

#ifndef DQDK_CEIL
#define DQDK_CEIL 0
#endif
#ifndef DQDK_NO_TOT  // (A/B timing only: the segment sizes not published; tables wrong)
#define DQDK_NO_TOT 0
#endif
#if DQDK_CEIL
// Timing-only CEILING of the fused decode's read + write pattern (VERDICT r5
// item 2; A/B builds only, -DDQDK_CEIL=1 or 2; the table comes out empty):
// the same phase A, load ring, windows, checksum sums and key arithmetic,
// but no LDS stage, no round flush and no round barrier.  A window's two
// keys (as fused_pair computes them) are packed to 16 bits each and the
// wave writes them with one streaming store per window to a region of its
// own: 256 contiguous bytes a window, against the shipped decode's 243 B of
// key triples per 1500 B frame (91 events x 8/3 B) written through the
// stage.  DQDK_CEIL=2 issues the same stores to an offset past the region
// (dropped: the arithmetic stays live, nothing is written).
__device__ __forceinline__ uint32_t ceil_keys(const u32x4& va, const u32x4& vb, uint32_t r, uint32_t e0, uint32_t Ef)
{
    uint32_t out = 0;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const u32x4& v = c ? vb : va;
        const uint32_t x = __builtin_amdgcn_alignbyte(v.y, v.x, r);
        const uint32_t y = __builtin_amdgcn_alignbyte(v.z, v.y, r);
        const uint32_t ch = x & 0xffffu;
        const uint32_t bin = __builtin_amdgcn_perm(y, x, 0x0c0c0403u);
        const uint32_t hc = __builtin_amdgcn_ubfe(y, 16, 3);
        const uint32_t key = __umul24(ch, kHists << 16) + (hc << 16) + bin;
        const bool ink = e0 + 64u * c < Ef && ch < kChannels && hc < kHists;
        out |= (ink ? (key ^ (key >> 16)) & 0xffffu : 0u) << (16 * c);
    }
    return out;
}
#endif

// Phase A's keys (akey[0, na), KEY_NONE: out of bounds) into the stage, as
// fused_pair stages a window's: every returning LDS add first (lanes with
// no key add to their sink word), one wait, then the stores, then one
// ballot for the rare overflow -- one LDS round trip, not kAEv.
__device__ __forceinline__ void fused_keys_a(const RxArgs& a, const uint32_t (&akey)[kAEv], uint32_t na,
                                             uint32_t oob_slot, FusedLds& lds, __amdgpu_buffer_rsrc_t ovf_rsrc,
                                             uint32_t lane)
{
    uint32_t* const sink = &lds.csink[lane];
    uint32_t sl[kAEv];
#pragma unroll
    for (int k = 0; k < kAEv; k++) {
        const bool has = (uint32_t)k < na, inb = akey[k] != DQDK_KEY_NONE;
        const uint32_t b = min(akey[k] >> kL1Shift, (uint32_t)kL1Buckets - 1);
        sl[k] = atomicAdd(has ? (inb ? &lds.scnt[b] : &lds.oob[oob_slot]) : sink, 1u);
    }
    bool anyov = false;
#pragma unroll
    for (int k = 0; k < kAEv; k++) {
        const bool ink = (uint32_t)k < na && akey[k] != DQDK_KEY_NONE;
        const uint32_t b = min(akey[k] >> kL1Shift, (uint32_t)kL1Buckets - 1);
        const bool st = ink && sl[k] < (uint32_t)kFCap;
        stage_key(lds, st, b, sl[k], akey[k], lane);
        anyov |= ink && !st;
    }
    if (__ballot(anyov)) {  // rare: overflow slots
#pragma unroll
        for (int k = 0; k < kAEv; k++) {
            const bool ov = (uint32_t)k < na && akey[k] != DQDK_KEY_NONE && sl[k] >= (uint32_t)kFCap;
            const uint64_t om = __ballot(ov);
            if (om) {
                const uint32_t first = (uint32_t)__builtin_ctzll(om);
                uint32_t base = 0;
                if (lane == first)
                    base = atomicAdd(&lds.ovf_n, (uint32_t)__builtin_popcountll(om));
                base = rdl(base, first);
                ovf_put(a, ovf_rsrc, akey[k], ov,
                        base + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(om >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)om, 0u)));
            }
        }
    }
}

// Append the round's staged runs to the block's pieces.  Wave w owns buckets
// w, w + kFWaves, ... (lane j: bucket w + kFWaves*j, its piece cursor `cur`,
// in keys).  The stage already holds the piece's format (three keys to a
// word), so a run's words are copied unchanged.  A round flushes whole words
// (lines policy: whole 128-B lines, 16 words) and carries the rest (at most
// one word; lines policy: at most 16) to the stage's start; the last flush
// writes everything (the fields past the run hold zero, or keys sent to the
// overflow region: the piece size marks the valid keys).  The buckets are
// written two at a time: lanes 0-31 take the words of bucket slot 2p, lanes
// 32-63 those of slot 2p + 1, two words (one LDS read, one 16-B store) per
// lane and an 8-B store for a run's odd last word -- runs of up to 64 words
// in one pass, longer ones (a stage nearly full) in a second, rare pass --
// through one buffer descriptor per pair with per-lane offsets.  Every store
// is issued (its offset dropped past the run): a fixed VMEM pattern.  The
// flushed words are zeroed for the next round's ORs.  Rare: keys past a full
// piece go to the block's overflow region (u32 keys, slot from an LDS
// counter).
template <bool kLines, bool kLast>
__device__ __forceinline__ void fused_flush(const RxArgs& a, FusedLds& lds, int lane, uint32_t wave, uint32_t& cur,
                                            __amdgpu_buffer_rsrc_t ovf_rsrc)
{
    constexpr bool last = kLast;
    const uint32_t b = wave + (uint32_t)kFWaves * (uint32_t)lane;
    uint32_t c = 0, w = 0, fit = 0;
    if (b < (uint32_t)kL1Buckets) {
        c = min(lds.scnt[b], (uint32_t)kFCap);
        // lines policy: whole 128-B lines of words (the piece cursor stays
        // line-aligned, so no store writes part of a line); else whole words
        w = last ? c : kLines ? c - c % kLineKeys : c - c % 3u;
        fit = min(w, a.piece_cap - cur);  // (cap and cur are multiples of 3: so is fit before the last flush)
    }
    const uint32_t nw = (fit + 2u) / 3u;           // words to the piece
    const uint32_t nz = last ? 0u : w / 3u;         // words flushed (to the piece or the overflow): zeroed
    // the lane's bucket: byte offset of its next word inside the bucket's
    // region (cur is a multiple of 3 before the last flush)
    const uint32_t cbo = blockIdx.x * a.piece_words * 4u + (cur / 3u) * 8u;
    constexpr int NJ = (kL1Buckets + kFWaves - 1) / kFWaves;  // 18 bucket slots per wave
    constexpr int NP = (NJ + 1) / 2;                          // 9 pairs
    constexpr int GP = 3;                                     // pairs per batch of LDS reads
    const uint32_t half = (uint32_t)lane >> 5, t = (uint32_t)lane & 31u;
    const uint32_t hoff = half * (uint32_t)kFWaves * (uint32_t)a.region * 4u;  // slot 2p + 1's bucket: 16 regions on
    const uint64_t pair_bytes = (uint64_t)(kFWaves + 1) * a.region * 4u;
    // rare: keys past a full piece (words [fit / 3, w / 3)) to the overflow
    // region, before their words are zeroed
    for (uint64_t m = __ballot(fit < w); m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint32_t bj = wave + (uint32_t)kFWaves * j;
        const uint32_t fj = rdl(fit, j), nov = rdl(w, j) - fj;  // (fj: a multiple of 3 unless last)
        uint32_t o = 0;
        if (lane == 0)
            o = atomicAdd(&lds.ovf_n, nov);
        o = rfl(o);
        for (uint32_t k = (uint32_t)lane; k < nov; k += 64) {
            const uint32_t s = fj + k, q = s / 3u;
            const uint32_t key = (uint32_t)(lds.stage[bj * (uint32_t)kFCapW + q] >> (kL1Shift * (s - 3u * q))) & kTripleMask;
            ovf_put(a, ovf_rsrc, (bj << kL1Shift) | key, true, o + k);
        }
    }
    const uint64_t anyf = __ballot(nw != 0 || nz != 0);
    // pair p, words [2 t0, 2 t0 + 64) of each run: LDS reads (v) / stores + zeroing
    auto rd = [&](int p, uint32_t t0, u64x2& v) {
        const uint32_t bj = min(wave + (uint32_t)kFWaves * ((uint32_t)(2 * p) + half), (uint32_t)kL1Buckets - 1);
        // (lanes past the run read the next bucket's words or the slack: unused)
        v = *(const u64x2*)&lds.stage[bj * (uint32_t)kFCapW + 2u * (t0 + t)];
    };
    auto st = [&](int p, uint32_t t0, const u64x2& v) {
        if (((anyf >> (2 * p)) & 3ull) == 0)
            return;  // (wave-uniform) nothing in the pair's buckets
        const uint32_t n0 = rdl(nw, 2 * p), n1 = 2 * p + 1 < NJ ? rdl(nw, 2 * p + 1) : 0u;
        const uint32_t c0 = rdl(cbo, 2 * p), c1 = 2 * p + 1 < NJ ? rdl(cbo, 2 * p + 1) : 0u;
        const uint32_t nj = half ? n1 : n0, cj = half ? c1 : c0;
        const uint32_t q = 2u * (t0 + t);  // the lane's first word
        const uint32_t bj0 = wave + (uint32_t)kFWaves * (uint32_t)(2 * p);
        const __amdgpu_buffer_rsrc_t prs = uniform_rsrc(a.part1 + (uint64_t)bj0 * a.region, pair_bytes);
        const uint32_t off = hoff + cj + q * 8u;
        const uint64_t w0 = v.x;
        constexpr int aux = kLines ? kFstAuxLines : kFstAux;
        __builtin_amdgcn_raw_buffer_store_b128(as_u32x4(v), prs, q + 2u <= nj ? off : kOOB, 0, aux);
        __builtin_amdgcn_raw_buffer_store_b64(as_u32x2(w0), prs, q + 1u == nj ? off : kOOB, 0, aux);
        if (!last) {  // the flushed words, for the next round's ORs
            const uint32_t z0 = rdl(nz, 2 * p), z1 = 2 * p + 1 < NJ ? rdl(nz, 2 * p + 1) : 0u;
            const uint32_t zj = half ? z1 : z0;
            const uint32_t bj = wave + (uint32_t)kFWaves * ((uint32_t)(2 * p) + half);
            if (q + 2u <= zj)
                *(u64x2*)&lds.stage[bj * (uint32_t)kFCapW + q] = u64x2{0ull, 0ull};
            else if (q + 1u == zj)
                lds.stage[bj * (uint32_t)kFCapW + q] = 0ull;
        }
    };
#pragma unroll 1
    for (int h = 0; h < NP; h += GP) {
        u64x2 v[GP];
#pragma unroll
        for (int g = 0; g < GP; g++)
            if (h + g < NP)
                rd(h + g, 0u, v[g]);
#pragma unroll
        for (int g = 0; g < GP; g++)
            if (h + g < NP)
                st(h + g, 0u, v[g]);
    }
    // runs past 64 words: a second pass per such pair (never in the lines
    // policy's rounds, which flush at most two 16-word lines of a bucket)
    if (!kLines || kLast) {
        uint64_t m = __ballot(nw > 64u || nz > 64u);
        while (m) {
            const int p = (int)__builtin_ctzll(m) >> 1;
            m &= ~(3ull << (2 * p));  // (both slots of the pair at once)
            u64x2 v;
            rd(p, 32u, v);
            st(p, 32u, v);
        }
    }
    // carry the remainders to the stage's start (words [w / 3, ceil(c / 3)):
    // behind the flushed ones, so source and destination do not overlap)
    if (!last) {
        if (kLines) {  // up to 16 words: a wave per bucket
            for (uint64_t m = __ballot(w != 0 && c > w); m; m &= m - 1) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                const uint32_t bj = wave + (uint32_t)kFWaves * j;
                const uint32_t wj = rdl(w, j) / 3u, r = (rdl(c, j) + 2u) / 3u - wj;
                uint64_t* const sg = &lds.stage[bj * (uint32_t)kFCapW];
                uint64_t x = 0;
                if ((uint32_t)lane < r)
                    x = sg[wj + lane];
                if ((uint32_t)lane < r) {
                    sg[lane] = x;
                    sg[wj + lane] = 0ull;
                }
            }
        } else if (w != 0 && c > w) {  // one word: each lane its own bucket
            uint64_t* const sg = &lds.stage[b * (uint32_t)kFCapW];
            const uint64_t x = sg[w / 3u];
            sg[0] = x;
            sg[w / 3u] = 0ull;
        }
    }
    if (b < (uint32_t)kL1Buckets) {
        cur += fit;
        lds.scnt[b] = c - w;
    }
}

// Two policies for the pieces' partial lines (runs end mid-line), chosen by
// the host per frame density:
//   kLdAux  the frame loads' cache policy: 2 = non-temporal (the frames are
//           read once; out of L2 they leave it to the partial lines, which
//           the next round completes there);
//   kLines  flush whole 128-B lines only, carrying each bucket's remainder
//           (< 32 keys) to the next round: no partial line is ever written.
//   kHeadA  phase A decodes the events (and sums the checksum bytes) of each
//           frame's first cache line, which it read for the headers; the
//           stream starts after them (frame_geo's a_end)
template <int kLdAux, bool kLines, bool kHeadA>
__global__ void __launch_bounds__(kFThreads, 1) rx_decode_fused_kernel(RxArgs a)
{
    __shared__ FusedLds lds;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wave = rfl((uint32_t)(tid >> 6));
    const uint32_t wslot0 = wave * 64;
    for (int b = tid; b < kL1Buckets + 4; b += kFThreads)
        lds.scnt[b] = 0;
    for (uint32_t q = (uint32_t)tid; q < (kStageWords + 64) / 2; q += kFThreads)  // the stage's words: zero
        ((u64x2*)lds.stage)[q] = u64x2{0ull, 0ull};
    lds.sum[tid] = 0;
    lds.oob[tid] = 0;
    if (tid == 0)
        lds.ovf_n = 0;
    if (tid < kFoldWords)
        lds.fc[tid] = tid == F_FAIL ? ~0u : 0u;
    __syncthreads();
    // this block's private overflow region (ovf_blk_cap keys, then the table)
    uint32_t* const ovf_blk = a.ovf_blk + (uint64_t)blockIdx.x * a.ovf_blk_cap;
    const __amdgpu_buffer_rsrc_t ovf_rsrc = uniform_rsrc(ovf_blk, (uint64_t)a.ovf_blk_cap * 4u);
    // per-batch state reset -- with the counters folded, the last block's
    // fold_publish writes every one of these words instead: two blocks' plain
    // stores to one line, on different XCDs (each its own L2), would leave
    // the value to whichever L2 writes back last (advisor, round 4)
    if (!a.fold && blockIdx.x == 0 && tid < 17)
        a.batch_scratch[tid] = tid == 0 ? (uint64_t)a.n : 0ull;

    const uint32_t ntiles = (a.n + 63) / 64;
    const uint32_t nsuper = (ntiles + kFWaves - 1) / kFWaves;
    const int W = (int)a.round_windows;
    uint32_t fcur = 0;  // the piece cursor of this lane's bucket (wave + kFWaves * lane)
    int kr = 0;         // windows of the current round so far: rounds run on across super-tiles
#if DQDK_CEIL
    // the ceiling's per-wave output region (1 KiB-aligned share of the pieces' allocation)
    const uint64_t ceil_words =
        ((uint64_t)kL1Buckets * a.region / ((uint64_t)gridDim.x * kFWaves)) & ~(uint64_t)255;
    const __amdgpu_buffer_rsrc_t ceil_rsrc =
        uniform_rsrc(a.part1 + ((uint64_t)blockIdx.x * kFWaves + wave) * ceil_words, ceil_words * 4u);
    uint32_t ceil_off = (uint32_t)lane * 4u;
#endif
    for (uint32_t st = blockIdx.x; st < nsuper; st += gridDim.x) {
        const uint32_t tile = st * kFWaves + wave;
        // frame of this lane: tile-major (64 consecutive frames per wave), or
        // interleaved (a.fmap: the block's waves stream 16 adjacent frames at
        // a time -- lane l of wave w takes frame 1024 st + 16 l + w)
        const uint32_t i = a.fmap ? st * (64u * kFWaves) + (uint32_t)lane * kFWaves + wave : tile * 64 + (uint32_t)lane;
        const bool live = i < a.n;

        // ---- phase A ----
        FrameInfo fi;
        dqdk_gpu_rx_result_t r;
        LaneFrame lf;
        bool stream;
        uint32_t akey[kAEv], na, hw;
        phase_a<kHeadA>(a, i, live, fi, r, lf, stream, akey, na, hw);
        (void)hw;
        if (kHeadA && __ballot(na != 0)) {
            // (mid-round: rounds run on across super-tiles; keys past a
            // full stage go to the overflow region like any others)
            fused_keys_a(a, akey, na, wslot0 + (uint32_t)lane, lds, ovf_rsrc, (uint32_t)lane);
        }
        const uint64_t smask0 = __ballot(stream);
        const int total = smask0 ? (int)wave_sum_dpp(pk_nwin(lf.pk1)) : 0;
        if (lane == 0)
            lds.wtot[wave] = (uint32_t)total;
        lds_barrier();
        int tmax = 0;
#pragma unroll
        for (int w = 0; w < kFWaves; w++)
            tmax = max(tmax, (int)lds.wtot[w]);
        // the same for every wave: the barriers below match
        const int kend = (tmax + kFRingW - 1) / kFRingW * kFRingW;
        lds_barrier();  // wtot is rewritten by the next super-tile

        // ---- phase B: rounds of W windows, the block's stage flushed after each ----
        const uint32_t lane16 = (uint32_t)lane * 16u;
        uint64_t lmask = smask0;
        uint32_t jl = smask0 ? (uint32_t)__builtin_ctzll(lmask) : 0u;
        uint32_t wl = 0, lnwin = smask0 ? pk_nwin(rdl(lf.pk1, jl)) : 0u;
        __amdgpu_buffer_rsrc_t lrs = frame_rsrc(lf, jl);
        // (kHeadA) lane 0 of a sh frame's first window loads 4 B further: its
        // chunk's first dword lies in the line phase A read (PFrame::hw)
        const uint32_t lsh_lane = kHeadA && lane == 0 ? 4u : 0u;
        uint32_t lsh = kHeadA && smask0 ? (rdl(lf.pk2, jl) >> 27) & 1u : 0u;
        auto issue = [&](u32x4& d0, u32x4& d1) {
            const uint32_t vo = lane16 + (lmask != 0 ? wl * kWinBytes + (wl == 0 && lsh ? lsh_lane : 0u) : kOOB);
            d0 = __builtin_amdgcn_raw_buffer_load_b128(lrs, vo, 0, kLdAux);
            d1 = __builtin_amdgcn_raw_buffer_load_b128(lrs, vo + 1024u - (wl == 0 && lsh ? lsh_lane : 0u), 0, kLdAux);
            if (lmask != 0 && ++wl == lnwin) {
                wl = 0;
                lmask &= lmask - 1;
                if (lmask) {
                    jl = (uint32_t)__builtin_ctzll(lmask);
                    lnwin = pk_nwin(rdl(lf.pk1, jl));
                    lrs = frame_rsrc(lf, jl);
                    if (kHeadA)
                        lsh = (rdl(lf.pk2, jl) >> 27) & 1u;
                }
            }
        };
        u32x4 b0[kFRingW], b1[kFRingW];
#pragma unroll
        for (int d = 0; d < kFRingW; d++)
            issue(b0[d], b1[d]);
        uint64_t pmask = smask0;
        uint32_t jp = smask0 ? (uint32_t)__builtin_ctzll(pmask) : 0u;
        uint32_t wp = 0;
        PFrame P;
        auto pfr = [&](uint32_t j) { pframe(a, lf, j, P); };
        if (smask0)
            pfr(jp);
        else
            P = PFrame{0, 0, 0, 0, 0, 0, 0, kNoWin, kNoWin, 0, 16};
        uint32_t acc0 = 0, acc1 = 0;
        // one loop over the super-tile's windows (a flush inside it every W
        // windows of the block's count, which runs on across super-tiles):
        // a single back-edge keeps the compiler's vmcnt accounting of the
        // load ring exact across rounds
        for (int k = 0; k < kend; k += kFRingW) {
#pragma unroll
            for (int d = 0; d < kFRingW; d++) {
                const bool active = k + d < total;
                const uint32_t jw = (uint32_t)kWinChunks * wp;
                if (kHeadA && active && wp == 0 && P.sh && lane == 0)  // the frame's first chunk: hw + 12 loaded bytes
                    b0[d] = u32x4{P.hw, b0[d].x, b0[d].y, b0[d].z};
                if (active && wp >= P.mw) {
                    const int j0 = (int)jw + lane;
                    csum_pair(b0[d], b1[d], j0 <= P.ct ? u16x2{1, 1} : u16x2{0, 0},
                              j0 + 64 <= P.ct ? u16x2{1, 1} : u16x2{0, 0}, acc0, acc1);
                } else {
                    csum_pair(b0[d], b1[d], u16x2{1, 1}, u16x2{1, 1}, acc0, acc1);
                }
                if (active && wp == P.tw) {  // (wave-uniform) the frame's last checksum chunk
                    // its bytes past the datagram leave the sum here, by the
                    // lane holding it (no per-frame LDS copy for phase C)
                    if (lane == (int)P.tl) {
                        if (P.th)
                            acc1 -= tail_corr(b1[d], (int)P.keep);
                        else
                            acc0 -= tail_corr(b0[d], (int)P.keep);
                    }
                }
                const uint32_t Ef = active ? P.Ef : 0u;
                const uint32_t e0 = jw + (uint32_t)lane - P.de;
#if DQDK_CEIL
                {
                    const uint32_t cw = ceil_keys(b0[d], b1[d], P.r, e0, Ef);
                    __builtin_amdgcn_raw_buffer_store_b32(cw, ceil_rsrc, DQDK_CEIL == 1 && active ? ceil_off : kOOB,
                                                          0, kFstAuxLines);
                    ceil_off += active ? 256u : 0u;
                }
#else
                fused_pair(a, b0[d], b1[d], P.r, e0, Ef, wslot0 + jp, lds, ovf_rsrc, (uint32_t)lane);
#endif
                if (active && ++wp == P.nwin) {
                    frame_sum_add(&lds.sum[wslot0 + jp], &lds.csink[lane], acc0 + acc1,
                                  (lane & 15) == 15);
                    acc0 = acc1 = 0;
                    wp = 0;
                    pmask &= pmask - 1;
                    if (pmask) {
                        jp = (uint32_t)__builtin_ctzll(pmask);
                        pfr(jp);
                    }
                }
                issue(b0[d], b1[d]);
            }
            kr += kFRingW;
            if (!DQDK_CEIL && kr == W) {  // end of a round (block-uniform)
                kr = 0;
                lds_barrier();
                fused_flush<kLines, false>(a, lds, lane, wave, fcur, ovf_rsrc);
                lds_barrier();
            }
        }

        // ---- phase C ----
        const uint32_t my = wslot0 + (uint32_t)lane;
        const uint32_t sum_t = lds.sum[my], sum_oob = lds.oob[my];
        lds.sum[my] = 0;
        lds.oob[my] = 0;
        phase_c(a, i, live, stream, fi, r, sum_t, sum_oob, u32x4{0u, 0u, 0u, 0u});
        if (a.fold)
            fold_frames(a, lds.fc, live, r, i, lane);
        // decoded, then failed the UDP checksum: its keys are staged already,
        // so the wave takes their events back from the table now (rare)
        for (uint64_t fm = __ballot(live && (fi.work & 1) && r.status != DQDK_RX_OK); fm; fm &= fm - 1)
            takeback_frame(a, rdl(i, (uint32_t)__builtin_ctzll(fm)), (uint32_t)lane);
    }
    // the keys still staged, then the piece sizes for rx_part1 / rx_part2
    lds_barrier();
    if (!DQDK_CEIL)
        fused_flush<kLines, true>(a, lds, lane, wave, fcur, ovf_rsrc);
    {
        // this block's piece sizes, and (device atomics, executed at the
        // memory side: no fence) their triples per bucket, rx_part2's segment sizes
        const uint32_t b = wave + (uint32_t)kFWaves * (uint32_t)lane;
        if (b < (uint32_t)kL1Buckets) {
            a.scratch[kOffPieceN + b * kMaxFusedGrid + blockIdx.x] = fcur;
            if (fcur && !DQDK_NO_TOT)
                __hip_atomic_fetch_add(&a.scratch[kOffPieceTotT + b * kTotStride], (fcur + 2u) / 3u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the block's private overflow region is appended to the overflow list
    __syncthreads();  // (also orders the region's stores before the copy below)
    // (the last flush left every stage count at 0: they count the region's
    // keys per bucket here, then one device atomic per bucket per block)
    const uint32_t nov = min(lds.ovf_n, a.ovf_blk_cap);  // (the keys past the region went to the table)
    if (nov && !a.ovf_list) {
        // each key to the table's base plane by a relaxed device atomic (the
        // reference's ++ at src/tristan.c:243); the count, for the host's
        // choice of the next batches' form (rx_part2 reports it)
        if (tid == 0)
            atomicAdd(&a.scratch[kOffOvfN], nov);
        for (uint32_t t = (uint32_t)tid; t < nov; t += kFThreads)
            __hip_atomic_fetch_add(&a.hist[ovf_blk[t]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (nov) {
        // the list form (after a batch with a long list): rx_part1 groups it
        // by bucket for rx_part2
        if (tid == 0)
            lds.wtot[0] = atomicAdd(&a.scratch[kOffOvfN], nov);
        __syncthreads();
        const uint32_t o = lds.wtot[0];
        for (uint32_t t = (uint32_t)tid; t < nov; t += kFThreads) {
            const uint32_t k = ovf_blk[t];
            a.ovf[o + t] = k;
            atomicAdd(&lds.scnt[k >> kL1Shift], 1u);
        }
        __syncthreads();
        if (tid < kL1Buckets && lds.scnt[tid])
            atomicAdd(&a.scratch[kOffCnt1 + tid], lds.scnt[tid]);
    }
    if (a.fold)
        fold_publish(a, lds.fc, tid);
}

// the shipped variants (fused_policy_default: 3 from 128 events per frame,
// else 2); the A/B build (-DDQDK_AB_VARIANTS) holds the other six as well
template __global__ void rx_decode_fused_kernel<2, false, false>(RxArgs);
template __global__ void rx_decode_fused_kernel<2, true, false>(RxArgs);
#ifdef DQDK_AB_VARIANTS
template __global__ void rx_decode_fused_kernel<0, false, false>(RxArgs);
template __global__ void rx_decode_fused_kernel<0, true, false>(RxArgs);
template __global__ void rx_decode_fused_kernel<0, false, true>(RxArgs);
template __global__ void rx_decode_fused_kernel<0, true, true>(RxArgs);
template __global__ void rx_decode_fused_kernel<2, false, true>(RxArgs);
template __global__ void rx_decode_fused_kernel<2, true, true>(RxArgs);
#endif

// ---------------------------------------------------------------------------
// Counters (fetch_xsk accounting, src/dqdk.c:252-322; tristan.c:327-328).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool in_batch(uint32_t st)
{
    return st != DQDK_RX_FILTER_DROP && st != DQDK_RX_FILTER_PASS;
}

constexpr int kAbortLoads = 8;  // result loads in flight per thread (independent: no break between them)

__device__ __forceinline__ void abort_block(const CountArgs& a)
{
    uint64_t m = a.n;
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < a.n && m == a.n; i0 += kAbortLoads * stride) {
        uint32_t st[kAbortLoads];
#pragma unroll
        for (int u = 0; u < kAbortLoads; u++) {
            const uint32_t i = i0 + (uint32_t)u * stride;
            st[u] = i < a.n ? a.res[i].status : (uint32_t)DQDK_RX_OK;
        }
#pragma unroll
        for (int u = kAbortLoads - 1; u >= 0; u--)  // grid-stride order: the smallest failing i of this thread
            if (in_batch(st[u]) && st[u] != DQDK_RX_OK)
                m = i0 + (uint32_t)u * stride;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t x = __shfl_xor(m, o);
        m = x < m ? x : m;
    }
    if ((threadIdx.x & 63) == 0 && m < a.n)
        atomicMin((unsigned long long*)&a.batch_scratch[0], (unsigned long long)m);
}

__global__ void __launch_bounds__(256) rx_abort_kernel(CountArgs a) { abort_block(a); }

enum { C_FRAMES, C_PKTS, C_BYTES, C_IP, C_UDP, C_EVENTS, C_TBYTES, C_OOB, C_EMPTY, C_FILT, C_N };

__device__ __forceinline__ void count_block(const CountArgs& a)
{
    __shared__ uint64_t red[C_N][4];
    const uint64_t abort_idx = __hip_atomic_load(&a.batch_scratch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t limit = (a.flags & DQDK_GPU_F_BATCH_ABORT) ? (abort_idx < a.n ? abort_idx + 1 : a.n) : a.n;
    uint64_t c[C_N];
#pragma unroll
    for (int k = 0; k < C_N; k++)
        c[k] = 0;
    auto count = [&](uint32_t i, const dqdk_gpu_rx_result_t& r) {
        const uint32_t st = r.status;
        if (!in_batch(st)) {
            c[C_FILT]++;
            return;
        }
        c[C_FRAMES]++;
        if (i >= limit)
            return;
        c[C_PKTS]++;
        c[C_IP] += (st == DQDK_RX_INVALID_IP || st == DQDK_RX_INVALID_IP_CSUM);
        c[C_UDP] += (st == DQDK_RX_INVALID_UDP || st == DQDK_RX_INVALID_UDP_CSUM);
        c[C_EMPTY] += (st == DQDK_RX_EMPTY);
        if (st == DQDK_RX_OK) {
            c[C_BYTES] += r.datalen;
            c[C_TBYTES] += r.datalen;
            c[C_EVENTS] += a.E;
            c[C_OOB] += a.histo ? r.oob_events : 0u;
        }
    };
    // one block per CU (few blocks: every block ends in 20 device atomics on
    // the same 20 words), sixteen result loads in flight per thread (a 1M-frame
    // batch in one round trip)
    constexpr int kU = 16;
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < a.n; i0 += kU * stride) {
        uint2 r[kU];
#pragma unroll
        for (int u = 0; u < kU; u++)
            r[u] = i0 + u * stride < a.n ? *(const uint2*)&a.res[i0 + u * stride] : make_uint2(0u, 0xffu);
#pragma unroll
        for (int u = 0; u < kU; u++)
            if (i0 + u * stride < a.n) {
                count(i0 + u * stride, __builtin_bit_cast(dqdk_gpu_rx_result_t, r[u]));
                if (a.out_res)  // the host drop-in's per_pkt, straight into pinned host memory
                    ((uint2*)a.out_res)[i0 + u * stride] = r[u];
            }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < C_N; k++) {
        uint64_t v = c[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v += __shfl_xor(v, o);
        if (lane == 0)
            red[k][wave] = v;
    }
    __syncthreads();
    if (threadIdx.x < C_N) {
        const int k = threadIdx.x;
        const uint64_t v = red[k][0] + red[k][1] + red[k][2] + red[k][3];
        if (v) {
            unsigned long long* b = (unsigned long long*)&a.batch_scratch[1];
            unsigned long long* cum = (unsigned long long*)a.cum;
            const int slot = k < C_EVENTS ? k : k + 1;  // dqdk_gpu_counters_t order (skip failing_batches)
            atomicAdd(&b[slot], (unsigned long long)v);
            atomicAdd(&cum[slot], (unsigned long long)v);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long* b = (unsigned long long*)&a.batch_scratch[1];
        unsigned long long* cum = (unsigned long long*)a.cum;
        const unsigned long long failed = abort_idx < a.n ? 1ull : 0ull;
        if (failed) {
            atomicAdd(&b[5], failed);    // failing_batches
            atomicAdd(&cum[5], failed);
        }
        b[11] = abort_idx;               // first_abort_idx of this batch
        cum[11] = abort_idx;
    }
    if (a.out_batch) {
        // the last block to finish publishes the batch's counters to the host
        __shared__ uint32_t last;
        __threadfence();  // this block's counter adds (and block 0's stores) before its ticket
        __syncthreads();
        if (threadIdx.x == 0)
            last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
        __syncthreads();
        if (last) {
            __threadfence();
            if (threadIdx.x < kBatchOut)
                a.out_batch[threadIdx.x] =
                    __hip_atomic_load(&a.batch_scratch[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (threadIdx.x == 0)
                *a.ticket = 0;
        }
    }
    if (a.out_res || a.out_batch)
        __threadfence_system();  // host-memory writes visible once the kernel completes
}

__global__ void __launch_bounds__(256) rx_count_kernel(CountArgs a) { count_block(a); }

// A batch of at most kTile frames in one launch: the decode (records path),
// then this block's own rx_abort and rx_count over the results it just
// wrote -- one launch instead of three for DQDK's small RX batches (-b 64,
// src/tristan.c:393), where the launches are the call's latency.
__global__ void __launch_bounds__(kTile) rx_small_kernel(RxArgs ra, CountArgs ca)
{
    __shared__ DecodeLds lds;
    decode_block(ra, lds);
    __threadfence();  // the results and the batch-state reset, before the block reads them back
    __syncthreads();
    abort_block(ca);
    __threadfence();
    __syncthreads();
    count_block(ca);
}

// ---------------------------------------------------------------------------
// Histogram accumulation (src/tristan.c:233-245, :243 relaxed atomic ++).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t frames_limit(const HistoArgs& a)
{
    const uint64_t abort_idx = a.batch_scratch[0];
    return (a.flags & DQDK_GPU_F_BATCH_ABORT) ? (uint32_t)(abort_idx < a.n ? abort_idx : a.n) : a.n;
}

// Small batches: one relaxed agent-scope atomic per event, one wave per frame.
__global__ void __launch_bounds__(256) rx_histo_atomic_kernel(HistoArgs a)
{
    const uint32_t limit = frames_limit(a);
    const int lane = threadIdx.x & 63;
    const uint32_t gw = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t nw = (gridDim.x * 256) >> 6;
    for (uint32_t i = gw; i < limit; i += nw) {
        if (a.res[i].status != DQDK_RX_OK)
            continue;
        const uint32_t* k = a.keys + (uint64_t)i * a.E;
        for (uint32_t e = lane; e < a.E; e += 64) {
            const uint32_t key = k[e];
            if (key != DQDK_KEY_NONE)
                __hip_atomic_fetch_add(&a.hist[key], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Exclusive scan of src[0..n) (n <= 320) into dst[0..n], dst[n] = total, by
// wave 0 of the block (5 entries per lane).  Caller syncs afterwards.
__device__ __forceinline__ void wave0_excl_scan(const uint32_t* src, uint32_t* dst, int n, bool src_global,
                                                uint32_t align = 1)
{
    if (threadIdx.x >= 64)
        return;
    const int lane = threadIdx.x;
    uint32_t v[5], sum = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const int i = lane * 5 + j;
        v[j] = i < n ? (src_global ? __builtin_nontemporal_load(&src[i]) : src[i]) : 0u;
        v[j] = (v[j] + align - 1) & ~(align - 1);
        sum += v[j];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= o)
            incl += t;
    }
    uint32_t run = incl - sum;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const int i = lane * 5 + j;
        if (i <= n)
            dst[i] = run;
        run += v[j];
    }
}

// largest b with off[b] <= p, off[0] = 0, off monotone, b < nb
__device__ __forceinline__ int find_run(const uint32_t* off, int nb, uint32_t p)
{
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= p)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

#ifndef DQDK_P1_PIPE
#define DQDK_P1_PIPE 1
#endif
constexpr bool kP1Pipe = DQDK_P1_PIPE;  // part1 loads chunk c+1 while chunk c is written out

// Level 1: keys (frame order) -> part1, grouped by bucket = key >> 21.
// A block stages kP1Chunk keys in LDS sorted by bucket, reserves each
// bucket's run with one global atomic, and writes the runs out
// contiguously.  The keys of a thread are dword buffer loads issued back to
// back (lane-contiguous, out-of-range lanes read 0 and are dropped by
// index); the counting atomic returns each key's rank inside its bucket, so
// the scatter is a plain LDS store; the run reservations (284 returning
// atomics on 284 shared cursors, the contended step) are waited for only
// after the scatter.  One 32K-key chunk per block (128 KB of LDS, one block
// per CU) halves the reservations per key of a 16K chunk and doubles the
// average run written per bucket.
__global__ void __launch_bounds__(kP1Threads, kP1MinWaves) rx_part1_kernel(HistoArgs a)
{
    __shared__ uint32_t stage[kP1Chunk];
    __shared__ uint32_t off1[kL1Buckets + 1];
    __shared__ uint32_t lcnt[kL1Buckets];
    __shared__ uint32_t loff[kL1Buckets + 1];
    __shared__ uint32_t gdel[kL1Buckets];  // global position - LDS position of each bucket's run
    const int tid = threadIdx.x;
    // records path: the frame-order records of the accounted frames; fused
    // path: the decode's overflow list (usually empty)
    const uint32_t total = a.total_keys ? *a.total_keys : frames_limit(a) * a.E;
    if (a.fused && total <= kOvfAtomicMax) {
        // a short overflow list goes straight to the table's base plane, one
        // relaxed atomic per key (the reference's ++ at src/tristan.c:243):
        // grouped, each bucket holding a few of its keys would cost rx_part2
        // an item of its own
        for (uint32_t k = blockIdx.x * kP1Threads + tid; k < total; k += gridDim.x * kP1Threads)
            __hip_atomic_fetch_add(&a.hist[a.keys[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (total <= blockIdx.x * (uint32_t)kP1Chunk)
        return;  // no chunk for this block
    uint32_t* const out = a.part1 + a.part1_base;
    const uint32_t step = gridDim.x * (uint32_t)kP1Chunk;
    uint32_t* cur1 = a.scratch + kOffCur1;
    constexpr int kOwn = (kL1Buckets + kP1Threads - 1) / kP1Threads;  // buckets reserved per thread (1)
    wave0_excl_scan(a.scratch + kOffCnt1, off1, kL1Buckets, true, kBucketAlign);
    uint32_t key[kP1Keys];
    auto load = [&](uint32_t b0) {
        const uint32_t n0 = min(total - b0, (uint32_t)kP1Chunk);
        const __amdgpu_buffer_rsrc_t src = uniform_rsrc(a.keys + b0, (uint64_t)n0 * 4u);  // keys = records or overflow list
#pragma unroll
        for (int j = 0; j < kP1Keys; j++)
            key[j] = __builtin_amdgcn_raw_buffer_load_b32(src, (uint32_t)tid * 4u, j * kP1Threads * 4, 0);
    };
    if (kP1Pipe && blockIdx.x * (uint32_t)kP1Chunk < total)
        load(blockIdx.x * (uint32_t)kP1Chunk);
    for (uint32_t base = blockIdx.x * (uint32_t)kP1Chunk; base < total; base += step) {
        const uint32_t nk = min(total - base, (uint32_t)kP1Chunk);
        if (!kP1Pipe)
            load(base);
        for (int b = tid; b < kL1Buckets; b += kP1Threads)
            lcnt[b] = 0;
        __syncthreads();
        uint32_t rank[kP1Keys / 2];  // two u16 ranks per word (rank < kP1Chunk <= 65536)
#pragma unroll
        for (int j = 0; j < kP1Keys; j++) {
            // non-OK frames already hold KEY_NONE; lanes past the chunk are dropped
            if (!((uint32_t)(j * kP1Threads + tid) < nk))
                key[j] = DQDK_KEY_NONE;
            const uint32_t r = key[j] != DQDK_KEY_NONE ? atomicAdd(&lcnt[key[j] >> kL1Shift], 1u) : 0u;
            rank[j / 2] = (j & 1) ? (rank[j / 2] | (r << 16)) : r;
        }
        __syncthreads();
        // the run reservations need only the counts: they go out before the
        // scan, so their latency overlaps the scan, a barrier and the scatter
        uint32_t g[kOwn];
#pragma unroll
        for (int o = 0; o < kOwn; o++) {
            const int b = tid + o * kP1Threads;
            g[o] = b < kL1Buckets && lcnt[b] ? atomicAdd(&cur1[b], lcnt[b]) : 0u;
        }
        wave0_excl_scan(lcnt, loff, kL1Buckets, false);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kP1Keys; j++)
            if (key[j] != DQDK_KEY_NONE)
                stage[loff[key[j] >> kL1Shift] + ((rank[j / 2] >> (16 * (j & 1))) & 0xffffu)] = key[j];
#pragma unroll
        for (int o = 0; o < kOwn; o++) {
            const int b = tid + o * kP1Threads;
            if (b < kL1Buckets)
                gdel[b] = off1[b] + g[o] - loff[b];
        }
        // the next chunk's keys load while this one is written out (key[] is
        // free once scattered)
        if (kP1Pipe && base + step < total)
            load(base + step);
        __syncthreads();
        const uint32_t nkeys = loff[kL1Buckets];
        for (uint32_t p = tid; p < nkeys; p += kP1Threads) {
            const uint32_t k = stage[p];
            out[p + gdel[k >> kL1Shift]] = k;
        }
        __syncthreads();
    }
}

// Level 2: each part2 item = one kPartChunk-key chunk of a segment, sorted by slice
// ((key >> 14) & 127) in LDS and written to part2 [item * kPartChunk, + keys) as u16
// (the key's low 16 bits: readers mask off bits 14-15, the slice's), with the
// run starts of its 128 slices.  A segment is a sequence of keys of one
// L1 bucket: records path, rx_part1's run of the bucket; fused path, the
// bucket's pieces (one per decode block, adjacent in the fused region,
// gathered through the scan of their sizes that rx_part1's prologue wrote),
// then rx_part1's run of the bucket's overflow keys.  Items are numbered
// segment by segment; every block derives the segment table and the item
// starts itself (a prologue over L2-resident counts, in place of a launch of
// its own), and block 0 publishes each bucket's first item for the slice pass.
//
// The item is a two-pass counting sort over per-lane-slot counters: slice s
// has 32 counters, cnt[s][l & 31], one per lane position of a 32-lane LDS
// group, so the 32 lanes of a group always add to 32 different banks (a
// random slice per lane over one counter per slice made 53 % of the LDS
// cycles bank conflicts and serialised same-slice adds: profiles/r04g).  Per
// key: one buffer load, one non-returning LDS add (count), a block-wide scan
// of the 4096 counters into run cursors (slice-major, so slice s's keys are
// the contiguous concatenation of its 32 sub-runs; the order inside a slice
// run is immaterial to the slice pass), one returning LDS add on the
// key's cursor (its byte offset in the stage) and one u16 LDS store.  Slots
// past the item and triple pads are masked off (no stage slot).  The next
// item's keys load while this one is written out.  The barriers hand off LDS
// data only (global reads are read-only inputs, global writes are not read
// back by the block): lds_barrier() keeps the next item's key loads in flight
// across them.
template <int kLdAux>
#ifndef DQDK_P2_WAVES  // waves per SIMD the register budget is cut for (8: two blocks per CU, 64 VGPRs)
#define DQDK_P2_WAVES 8
#endif
__global__ void __launch_bounds__(kPartThreads, DQDK_P2_WAVES) rx_part2_kernel(HistoArgs a)  // 32 waves per CU
{
    constexpr int kMaxSeg = kL1Buckets * kSegsPerBucket;
    constexpr int kPWaves = kPartThreads / 64;
    constexpr int kJT = kPartKeysPerThread / 3;                      // triple loads per lane (gathered items)
    constexpr uint32_t kWaveKeys = (uint32_t)kPartChunk / kPWaves;     // 1152 key slots per wave
    constexpr uint32_t kWaveTriples = kWaveKeys / 3;                  // 384 triple slots per wave
    constexpr uint32_t kDummy = 1u << kL1Shift;  // a slot past the item or a triple's pad (no stage slot)
    constexpr int kCtr = kSubs * 32;             // counters: [slice][lane & 31]
    static_assert(kCtr == 4 * kPartThreads, "the scan takes four counters per thread");
    __shared__ __attribute__((aligned(16))) uint16_t stage[kPartChunk + 2];  // + the dummies' sink
    __shared__ __attribute__((aligned(16))) uint32_t cnt[kCtr];  // counts (x2: bytes), zero between items
    __shared__ __attribute__((aligned(16))) uint32_t cur[kCtr];  // run cursors (byte offsets in the stage)
    __shared__ uint32_t prt[2][kMaxFusedGrid + 1], prk[2][kMaxFusedGrid + 1];  // piece starts: triples, keys
    __shared__ uint32_t s_cnt[kMaxSeg], ist[kMaxSeg + 1];
    __shared__ uint32_t off1[kL1Buckets + 1];
    __shared__ uint32_t wsum[kPWaves];
    const int tid = threadIdx.x;
    const uint32_t lane = (uint32_t)tid & 63u, wave = rfl((uint32_t)tid >> 6);
    const bool fused = a.fused != 0;
    const uint32_t nseg = fused ? (uint32_t)kMaxSeg : (uint32_t)kL1Buckets;

    // ---- prologue: segments (size, input index) and their first items ----
    wave0_excl_scan(a.scratch + kOffCnt1, off1, kL1Buckets, true, kBucketAlign);
    ((u32x4_t*)cnt)[tid] = u32x4_t{0u, 0u, 0u, 0u};
    __syncthreads();
    uint32_t nit = 0;
    if ((uint32_t)tid < nseg) {
        const uint32_t b = fused ? (uint32_t)tid >> 1 : (uint32_t)tid;
        uint32_t c, per;
        if (!fused || (tid & 1)) {  // rx_part1's run of the bucket: keys
            c = a.scratch[kOffCur1 + b];
            per = kPartChunk;
        } else {                    // the bucket's pieces: key triples
            c = a.scratch[kOffPieceTotT + b * kTotStride];  // (the decode's blocks summed their pieces' triples)
            per = kPartTriples;
        }
        s_cnt[tid] = c;
        nit = (c + per - 1) / per;
    }
    const uint32_t incl = wave_incl_scan_dpp(nit);
    if (lane == 63)
        wsum[wave] = incl;
    __syncthreads();
    uint32_t woff = 0;
    for (uint32_t w = 0; w < wave; w++)
        woff += wsum[w];
    if ((uint32_t)tid <= nseg)
        ist[tid] = woff + incl - nit;
    __syncthreads();
    const uint32_t nitems = rfl(ist[nseg]);
    if (blockIdx.x == 0 && tid <= kL1Buckets)
        a.scratch[kOffIstart + tid] = ist[fused ? 2 * tid : tid];

    // ---- an item's geometry (wave-uniform): its segment is the number of
    // segment starts ist[1..nseg) at or below it (nine ballots) ----
    struct Item {
        uint32_t s0;     // first unit of the item in its segment (gathered: triples, else keys)
        uint32_t nu;     // units
        uint32_t b;      // bucket
        uint32_t base8;  // contiguous input index / kBucketAlign
        bool gath;       // fused pieces (else one contiguous run)
    };
    // (the lane-derived addresses are opaque to the compiler: hoisted out of
    // the item loop they would stay live, and spill, across it)
    auto geo = [&](uint32_t item) {
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t t = 0;
#pragma unroll
        for (int m = 0; m < (kMaxSeg + 63) / 64; m++) {
            const uint32_t k = 1u + ln + 64u * (uint32_t)m;
            t += (uint32_t)__builtin_popcountll(__ballot(k < nseg && ist[min(k, (uint32_t)kMaxSeg)] <= item));
        }
        Item g;
        g.gath = fused && !(t & 1u);
        const uint32_t per = g.gath ? (uint32_t)kPartTriples : (uint32_t)kPartChunk;
        g.s0 = (item - rfl(ist[t])) * per;
        g.nu = min(rfl(s_cnt[t]) - g.s0, per);
        g.b = fused ? t >> 1 : t;
        // (a contiguous run's input: rx_part1's run of the bucket, 8-key aligned)
        g.base8 = g.gath ? 0u : (uint32_t)((a.part1_base + rfl(off1[g.b])) / kBucketAlign) + g.s0 / kBucketAlign;
        return g;
    };
    // a gathered item: its bucket's piece starts, the exclusive scans of the
    // decode blocks' piece sizes in keys (prk) and key triples (prt), by wave
    // 0 (four pieces a lane, DPP scans) from the sizes the decode wrote --
    // in two halves: the sizes' load early (into registers), the scans and
    // LDS stores late, so the load's latency passes under the work between
    // (then a barrier before they are read)
    u32x4_t pcn = u32x4_t{0u, 0u, 0u, 0u};
    auto fetch_pieces = [&](const Item& g) {
        if (g.gath && wave == 0) {
            const uint32_t l = opaque(lane);
            pcn = *(const u32x4_t*)(a.scratch + kOffPieceN + g.b * kMaxFusedGrid + 4u * l);
        }
    };
    auto put_pieces = [&](const Item& g, int pb) {
        if (g.gath && wave == 0) {
            const uint32_t l = opaque(lane);
            uint32_t v[4] = {pcn.x, pcn.y, pcn.z, pcn.w}, sum = 0, sumt = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                v[i] = 4u * l + (uint32_t)i < a.fgrid ? v[i] : 0u;  // (rows past the grid: stale)
                sum += v[i];
                sumt += (v[i] + 2u) / 3u;
            }
            const uint32_t incl = wave_incl_scan_dpp(sum), inclt = wave_incl_scan_dpp(sumt);
            uint32_t run = incl - sum, runt = inclt - sumt;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t blk = 4u * l + (uint32_t)i;
                if (blk < a.fgrid) {
                    prk[pb][blk] = run;
                    prt[pb][blk] = runt;
                }
                run += v[i];
                runt += (v[i] + 2u) / 3u;
            }
            if (l == 63) {
                prk[pb][a.fgrid] = incl;
                prt[pb][a.fgrid] = inclt;
            }
        }
    };
    auto stage_pieces = [&](const Item& g, int pb) {
        fetch_pieces(g);
        put_pieces(g, pb);
    };
    // slots: gathered items, wave w takes the item's triples [384w, 384w +
    // 384), 64 per load (load j: triple 384w + 64j + lane -> keys 3j .. 3j + 2
    // of the lane); contiguous items, keys [1152w, 1152w + 1152), 64 per load
    // (a gathered item's triple j loads into nk[2j], nk[2j + 1] and is
    // unpacked into key[3j .. 3j + 2] by count()).  A gathered item's loads
    // are issued a phase early: they land in nk while the previous item is
    // scanned, scattered and written out; a contiguous item's 15 keys (rx_part1
    // runs, rare on the fused path) load into key once the previous item's
    // scatter has freed it (no registers for both).
    uint32_t key[kPartKeysPerThread], nk[2 * kJT];
    uint32_t pad = 0;  // gathered: bit 2j + i set = key 3j + 2 - i is a pad of its piece's last triple
    auto load = [&](const Item& g, int pb) {
        pad = 0;
        if (g.gath) {
            // triple q of bucket b's sequence lies in piece p (prt[p] <= q <
            // prt[p + 1]) at byte p * words * 4 + (q - prt[p]) * 8 of the
            // bucket's region.  Lane state: t = start of the next piece - the
            // lane's first triple, u = byte offset of that triple were it in
            // the lane's current piece (a load's offset is u + 512 j); the
            // state moves only where a load reaches a piece's last triple (a
            // wave does about once)
            const __amdgpu_buffer_rsrc_t src = uniform_rsrc(a.part1 + (uint64_t)g.b * a.region, a.region * 4u);
            const uint32_t* pt = prt[pb];
            const uint32_t* pk = prk[pb];
            const uint32_t q0w = g.s0 + wave * kWaveTriples;
            uint32_t ln = lane;
            asm volatile("" : "+v"(ln));
            uint32_t lo = 0;
#pragma unroll
            for (int m = 0; m < (kMaxFusedGrid + 63) / 64; m++) {
                const uint32_t k = 1u + ln + 64u * (uint32_t)m;
                lo += (uint32_t)__builtin_popcountll(
                    __ballot(k < a.fgrid && pt[min(k, (uint32_t)kMaxFusedGrid)] <= q0w));
            }
            const uint32_t q0 = q0w + ln;
            uint32_t pl = lo, nl = pt[lo + 1];
            int32_t t = (int32_t)(nl - q0);
            uint32_t u = lo * a.piece_words * 4u + (q0 - pt[lo]) * 8u;
#pragma unroll
            for (int j = 0; j < kJT; j++) {
                if (__ballot(t <= 64 * j + 1)) {  // a lane at its piece's last triple or past it
                    const uint32_t q = q0 + 64u * (uint32_t)j;
                    while (q >= nl && pl + 1 < a.fgrid) {
                        pl++;
                        const uint32_t cl = nl;
                        nl = pt[pl + 1];
                        t = (int32_t)(nl - q0);
                        u = pl * a.piece_words * 4u + (q0 - cl) * 8u;
                    }
                    if (q + 1u == nl) {  // the piece's last triple: its valid keys
                        const uint32_t vc = pk[pl + 1] - pk[pl] - 3u * (q - pt[pl]);
                        pad |= ((vc < 3u ? 1u : 0u) | (vc < 2u ? 2u : 0u)) << (2 * j);
                    }
                }
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(src, u, 512 * j, kLdAux);
                nk[2 * j] = v.x;
                nk[2 * j + 1] = v.y;
            }
        }
    };
    auto load_contig = [&](const Item& g) {
        const __amdgpu_buffer_rsrc_t src = uniform_rsrc(a.part1 + (uint64_t)g.base8 * kBucketAlign, (uint64_t)g.nu * 4u);
#pragma unroll
        for (int j = 0; j < kPartKeysPerThread; j++)
            key[j] = __builtin_amdgcn_raw_buffer_load_b32(src, (wave * kWaveKeys + lane) * 4u, j * 256, kLdAux);
    };
    // count: every key (bucket-local, 21 bits) raises its slice's counter of
    // the lane's slot, cnt[(key >> 14) & 127][lane & 31], by 2 (bytes of a
    // u16); the key becomes (counter byte address << 16) | its low 16 bits,
    // all that scatter() needs of it.  Slots past the item and pads add 0.
    auto count = [&](const Item& g) {
        if (g.gath) {
#pragma unroll
            for (int j = kJT - 1; j >= 0; j--) {
                const uint32_t x = nk[2 * j], y = nk[2 * j + 1];
                key[3 * j] = x & kTripleMask;
                key[3 * j + 1] = __builtin_amdgcn_alignbit(y, x, kL1Shift) & kTripleMask;
                key[3 * j + 2] = y >> (2 * kL1Shift - 32);
            }
            if (__ballot(pad != 0)) {
#pragma unroll
                for (int j = 0; j < kJT; j++) {
                    key[3 * j + 2] = (pad >> (2 * j)) & 1u ? kDummy : key[3 * j + 2];
                    key[3 * j + 1] = (pad >> (2 * j)) & 2u ? kDummy : key[3 * j + 1];
                }
            }
            if (wave * kWaveTriples + kWaveTriples > g.nu) {
                // (the lane term opaque: hoisted per j out of the item loop,
                // the compares' operands would stay live, and spill)
                uint32_t ln = lane;
                asm volatile("" : "+v"(ln));
                const int32_t lim = (int32_t)g.nu - (int32_t)(wave * kWaveTriples);
#pragma unroll
                for (int j = 0; j < kJT; j++) {
                    const bool v = (int32_t)ln < lim - 64 * j;
#pragma unroll
                    for (int i = 0; i < 3; i++)
                        key[3 * j + i] = v ? key[3 * j + i] : kDummy;
                }
            }
        } else {
            const bool tail = wave * kWaveKeys + kWaveKeys > g.nu;
            uint32_t ln = lane;
            asm volatile("" : "+v"(ln));
            const int32_t lim = (int32_t)g.nu - (int32_t)(wave * kWaveKeys);
#pragma unroll
            for (int j = 0; j < kPartKeysPerThread; j++)
                key[j] = !tail || (int32_t)ln < lim - 64 * j ? key[j] & kTripleMask : kDummy;
        }
        // a dummy adds 0 to its lane's counter of slice 0 (no branch) and is
        // marked by bit 31 for scatter()
        const uint32_t sub4 = (lane & 31u) << 2;
#pragma unroll
        for (int j = 0; j < kPartKeysPerThread; j++) {
            // slice * 128 + (lane & 31) * 4: the counter's byte address
            const uint32_t ca = ((key[j] >> (kSliceBits - 7)) & ((kSubs - 1) << 7)) | sub4;
            const uint32_t d = key[j] >> kL1Shift;  // 1: dummy
            __hip_atomic_fetch_add(&cnt[ca >> 2], 2u - 2u * d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            key[j] = __builtin_amdgcn_perm(ca, key[j], 0x05040100u) | (d << 31);  // ca.lo16 : key.lo16
            // (opaque: scatter() re-derives the counter and increment from the
            // key; kept live across the scan they would spill)
            asm volatile("" : "+v"(key[j]));
        }
    };
    // scan: the counters (slice-major) into run cursors, four per thread;
    // the counts are zeroed for the next item.  Returns the item's valid
    // keys; item's 129 run starts (u16 offsets) go to runs.
    auto scan = [&](uint32_t item) -> uint32_t {
        const u32x4_t c = ((const u32x4_t*)cnt)[tid];
        uint32_t z = 0;
        asm volatile("" : "+v"(z));  // (a zero vector hoisted out of the item loop spills)
        ((u32x4_t*)cnt)[tid] = u32x4_t{z, z, z, z};
        const uint32_t sum = c.x + c.y + c.z + c.w;
        const uint32_t incl = wave_incl_scan_dpp(sum);
        if (lane == 63)
            wsum[wave] = incl;
        lds_barrier();
        // the waves' totals, one per lane (16 unrolled reads held 32 registers)
        const uint32_t x = lane < (uint32_t)kPWaves ? wsum[opaque(lane) & (kPWaves - 1)] : 0u;
        const uint32_t woff = wave_sum_dpp(lane < wave ? x : 0u), tot = wave_sum_dpp(x);
        const uint32_t ex = woff + incl - sum;
        ((u32x4_t*)cur)[tid] = u32x4_t{ex, ex + c.x, ex + c.x + c.y, ex + c.x + c.y + c.z};
        uint16_t* const ro = a.runs + (uint64_t)item * kItemOffs;
        if ((tid & 7) == 0)
            ro[opaque((uint32_t)tid) >> 3] = (uint16_t)(ex / 2);
        if (tid == 0)
            ro[kSubs] = (uint16_t)(tot / 2);
        return tot / 2;
    };
    // scatter: each key's u16 to the stage at its counter's cursor (a
    // returning add); every add of a round of 8 is issued before the first
    // store that uses one.
    auto scatter = [&]() {
#ifndef DQDK_P2_SG
#define DQDK_P2_SG 4
#endif
        constexpr int kSG = DQDK_P2_SG;
        uint8_t* const st8 = (uint8_t*)stage;
#pragma unroll
        for (int h = 0; h < kPartKeysPerThread; h += kSG) {
            uint32_t o[kSG];
#pragma unroll
            for (int j = 0; j < kSG; j++)
                if (h + j < kPartKeysPerThread)
                    o[j] = __hip_atomic_fetch_add(&cur[(key[h + j] >> 18) & (kCtr - 1)], 2u - 2u * (key[h + j] >> 31),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
            for (int j = 0; j < kSG; j++)
                if (h + j < kPartKeysPerThread)  // a dummy's u16 goes to the sink past the stage
                    *(uint16_t*)(st8 + ((key[h + j] >> 31) ? (uint32_t)kPartChunk * 2u : o[j])) = (uint16_t)key[h + j];
        }
    };

    // The item loop keeps three barriers an item: item i's scan (its own
    // barrier), then B2 (cursors) -> scatter -> the next item's count and the
    // piece starts of the one after it -> B3 (stage, counts, piece starts)
    // -> read-out of item i and the loads of item i + 2.  Invariant at the
    // top: item's counts are complete in cnt, g is item + gridDim.x's
    // geometry, its triples loading (gathered: nk) with its piece starts in
    // prt[pb ^ 1].
    Item g{};
    int pb = 0;
    uint32_t item = blockIdx.x;
    if (item < nitems) {
        g = geo(item);
        stage_pieces(g, 0);
        lds_barrier();
        if (g.gath)
            load(g, 0);
        else
            load_contig(g);
        count(g);
        if (item + gridDim.x < nitems) {
            g = geo(item + gridDim.x);
            stage_pieces(g, 1);
        }
        lds_barrier();
        if (item + gridDim.x < nitems && g.gath)
            load(g, 1);
    }
    for (; item < nitems; item += gridDim.x, pb ^= 1) {
        const uint32_t nv = scan(item);
        lds_barrier();
        // item i + 2's geometry and piece starts (loads now, LDS stores
        // before the barrier: prt[pb], last read by the loads of item)
        const bool more = item + gridDim.x < nitems;
        const bool more2 = item + 2u * gridDim.x < nitems;
        Item g2{};
        if (more2) {
            g2 = geo(item + 2u * gridDim.x);
            fetch_pieces(g2);
        }
        scatter();
        if (more) {
            if (!g.gath)
                load_contig(g);  // (a contiguous item's keys go straight to key[], which the scatter freed)
            count(g);            // (the scan zeroed the counters)
        }
        if (more2) {
            g = g2;
            put_pieces(g, pb);
        }
        lds_barrier();
        // item i's valid keys go to part2 [i * kPartChunk, + nv) in 16-B stores
        // (the bytes past nv in the last store are never read)
        const u32x4_t* st4 = (const u32x4_t*)stage;
        u32x4_t* dst4 = (u32x4_t*)(a.part2 + (uint64_t)item * kPartChunk);
        // (streaming stores: the slice pass reads them batches later, and
        // dirty lines left in L2 would be written back under the next
        // batch's decode -- r05v: decode -3 %, part2 +1 % at 1500 B)
        for (uint32_t p = opaque((uint32_t)tid); p * 8u < nv; p += kPartThreads)
            __builtin_nontemporal_store(st4[p], &dst4[p]);
        // item i + 2's triples load while item i + 1 is scanned, scattered
        // and written out
        if (more2 && g.gath)
            load(g, pb);
        // (no barrier here: the stage is rewritten, and wsum and the cursors
        // re-read, only after the next item's scan barrier)
    }
    if (a.p2_ticket) {
        // every block read the counters in its prologue: the last one to
        // finish zeroes them for the slot's next batch (device atomics and
        // the zeroing stores are ordered by the kernel boundary for the
        // kernels that follow on the stream)
        __shared__ uint32_t p2_last;
        __syncthreads();
        if (tid == 0)
            p2_last = atomicAdd(a.p2_ticket, 1u) == gridDim.x - 1;
        __syncthreads();
        if (p2_last) {
            if (fused && a.ovf_out && tid == 0)  // the batch's overflow, for the host's list-or-atomics choice
                __hip_atomic_store(a.ovf_out, (uint64_t)a.scratch[kOffOvfN], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __syncthreads();  // (read before it is zeroed)
            for (int w = tid; w < kZeroWords; w += kPartThreads)
                a.scratch[w] = 0u;
            if (tid == 0)
                *a.p2_ticket = 0u;
        }
    }
}

template __global__ void rx_part2_kernel<0>(HistoArgs);
template __global__ void rx_part2_kernel<2>(HistoArgs);

// Level 3: one block per span of kSliceSpan (2) adjacent 16K-bin slices:
// within a part2 item their runs are adjacent, so one run of ~240 keys per
// item and span (a latency-bound gather: twice the bytes per load round of a
// one-slice block).  The run offsets of the bucket's items (<= kSliceThreads
// at a time) are staged in LDS first, so gathering a run is one dependent
// load, and each wave gathers three items at once; the span's 32 KB of the
// table's low-byte plane is loaded up front and read-modify-written once
// after the LDS histogram is complete, with carries of 256 into the u32 base
// plane (rare: one per 256 increments of a bin).
//
// The bins are packed u16 pairs (64 KB: two 1024-thread blocks per CU, 32
// waves, hide the gather latency).  A bin cannot pass 65535: the runs are counted in groups of at
// most 65280 events, and between two groups every bin's high byte is
// drained into the base plane (an LDS sweep; a global add only where a bin
// reached 256), so any number of staged batches and any spectrum -- hot
// bins included -- is counted in one pass.
struct SliceLds {
    uint32_t s_run[kSliceThreads];  // lo | hi << 16: the run [lo, hi) of item s_base (u16 offsets)
    uint32_t s_pin[kSliceThreads];  // inclusive prefix of the run lengths of the staged entries
    uint32_t s_base[kSliceThreads];
    uint8_t s_k[kSliceThreads];
    uint32_t b_i0[kSliceMaxSlots], b_end[kSliceMaxSlots];  // the bucket's first item / inclusive prefix of its items per staged batch
    uint32_t w_tot[kSliceThreads / 64];
    uint32_t total;
};
constexpr uint32_t kDrainCap = 0xffffu - 0xffu;  // events per group: bins hold <= 255 after a drain

constexpr uint32_t kSpanMask = ((uint32_t)kSliceSpan << kSliceBits) - 1;  // a key's bin in its block's span

__device__ __forceinline__ void slice_count(uint32_t* h, uint32_t k)
{
    atomicAdd(&h[k >> 1], 1u << ((k & 1u) << 4));
}

// The runs of one slice over every staged batch form one flat list of
// (batch, item) entries -- the bucket's items of batch 0, then of batch 1,
// ...; entries [e0, e0 + n) are staged in LDS by one round of loads
// (kSliceMaxSlots: rx_kernels.h)

// counters: u16 pairs (8192 words)
__device__ __forceinline__ void slice_histo(const HistoArgs& a, uint32_t s, uint32_t* h, SliceLds& sl)
{
    constexpr int kWords = (kSliceSpan << kSliceBits) / 2;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    constexpr int kWavesS = kSliceThreads / 64;
    s *= kSliceSpan;  // the span's first slice
    const uint32_t b = s / kSubs, sub = s % kSubs;
    // staged batch k: its scratch (bucket starts, item starts), u16 keys, run offsets
    auto sc = [&](uint32_t k) { return a.scratch + (uint64_t)k * a.scratch_stride; };
    auto runs = [&](uint32_t k) { return a.runs + (uint64_t)k * a.runs_stride; };
    // the bucket's items per staged batch and their running total (LDS:
    // registers would be 64 more)
    static_assert(kSliceMaxSlots == 32, "one wave scans the staged batches; locate() searches 2^5 of them");
    if (tid < 64) {
        uint32_t i0 = 0, n = 0;
        if ((uint32_t)tid < a.nslots) {
            i0 = sc(tid)[kOffIstart + b];
            n = sc(tid)[kOffIstart + b + 1] - i0;
        }
        const uint32_t end = wave_incl_scan_dpp(n);
        if (tid < kSliceMaxSlots) {
            sl.b_i0[tid] = i0;
            sl.b_end[tid] = end;
        }
    }
    if (tid == 0)
        sl.total = 0;
    u32x4_t* h4 = (u32x4_t*)h;
    for (int c = tid; c < kWords / 4; c += kSliceThreads)
        h4[c] = u32x4_t{0u, 0u, 0u, 0u};
    __syncthreads();
    const uint32_t nent = sl.b_end[kSliceMaxSlots - 1];
    if (nent == 0)
        return;
    // entry e (< nent) -> its batch k (the first whose running total passes
    // e: a binary search) and item
    auto locate = [&](uint32_t e, uint32_t& k, uint32_t& it) {
        uint32_t lo = 0, hi = kSliceMaxSlots - 1;
#pragma unroll
        for (int s2 = 0; s2 < 5; s2++) {  // 2^5 = kSliceMaxSlots candidates
            const uint32_t mid = (lo + hi) >> 1;
            if (sl.b_end[mid] > e)
                hi = mid;
            else
                lo = mid + 1;
        }
        k = lo;
        it = sl.b_i0[lo] + e - (lo ? sl.b_end[lo - 1] : 0u);
    };
    // entries [e0, e0 + ne) -> LDS: run bounds, item base, batch
    auto stage = [&](uint32_t e0, uint32_t ne) -> uint32_t {
        uint32_t mine = 0;
        if ((uint32_t)tid < ne) {
            uint32_t k, it;
            locate(e0 + (uint32_t)tid, k, it);
            const uint16_t* ro = runs(k) + (uint64_t)it * kItemOffs + sub;
            const uint32_t lo = ro[0], hi = ro[kSliceSpan];
            sl.s_run[tid] = lo | (hi << 16);
            sl.s_base[tid] = it;
            sl.s_k[tid] = (uint8_t)k;
            mine = hi - lo;
        }
        return mine;
    };
    // s_run..s_k are written below only after every thread has read b_end
    __syncthreads();
    // events of this slice = sum of its run lengths: from the first staged
    // chunk of entries when it holds them all (the usual case), else a pass
    // (later chunks first: each thread overwrites only its own LDS slot, and
    // chunk 0's entries must be the ones left staged)
    uint32_t mine = 0;
    for (uint32_t e0 = (uint32_t)kSliceThreads; e0 < nent; e0 += kSliceThreads)
        mine += stage(e0, min(nent - e0, (uint32_t)kSliceThreads));
    const uint32_t mine0 = stage(0, min(nent, (uint32_t)kSliceThreads));
    mine += mine0;
    if (mine)
        atomicAdd(&sl.total, mine);
    __syncthreads();
    const uint32_t total = sl.total;
    if (total == 0)
        return;  // no events for this slice: table untouched
    const uint64_t sb = (uint64_t)s << kSliceBits;
    u32x4_t* lo4 = (u32x4_t*)(a.lo + sb);
    constexpr int kLoPer = (kSliceSpan << kSliceBits) / 16 / kSliceThreads;  // 2 x 16 B per thread
    u32x4_t l[kLoPer];
#pragma unroll
    for (int j = 0; j < kLoPer; j++)
        l[j] = lo4[tid + j * kSliceThreads];
    // each wave gathers kNI items at once, kKG dwords (two keys) per lane per
    // item per pass (384 keys: a whole typical span run), so a block takes its
    // items in rounds of kNI * kWavesS; runs start at any key: dword loads
    // from the run's first even key, halves outside the run are dropped
#ifndef DQDK_SLICE_NI
#define DQDK_SLICE_NI 3
#endif
#ifndef DQDK_SLICE_KG
#define DQDK_SLICE_KG 3
#endif
    constexpr int kNI = DQDK_SLICE_NI;
    constexpr int kKG = DQDK_SLICE_KG;
    // packed bins: move every bin's high byte into the base plane (bins left
    // <= 255).  Thread t owns bins [16t, +16) and [16(t + kSliceThreads), +16) here
    // and in the final read-modify-write, so its plain global adds are ordered.
    auto drain = [&]() {
#pragma unroll
        for (int j = 0; j < kLoPer; j++) {
            const uint32_t b0 = 16u * (uint32_t)(tid + j * kSliceThreads);
            u32x4_t* hc = (u32x4_t*)(h + b0 / 2);
            const u32x4_t c0 = hc[0], c1 = hc[1];
            uint32_t w8[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
            uint32_t any = 0;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                uint32_t& w = w8[m];
                const uint32_t hw = w & 0xff00ff00u;
                if (hw) {
                    if (hw & 0xffffu)
                        a.hist[sb + b0 + 2 * m] += hw & 0xffffu;
                    if (hw >> 16)
                        a.hist[sb + b0 + 2 * m + 1] += hw >> 16;
                    w &= 0x00ff00ffu;
                }
                any |= hw;
            }
            if (any) {
                hc[0] = u32x4_t{w8[0], w8[1], w8[2], w8[3]};
                hc[1] = u32x4_t{w8[4], w8[5], w8[6], w8[7]};
            }
        }
    };
    const bool drains = total > kDrainCap;  // else one group: no bin can pass 65535
    uint32_t since = 0;  // events counted since the last drain (block-uniform)
    for (uint32_t e0 = 0; e0 < nent; e0 += kSliceThreads) {
        const uint32_t nit = min(nent - e0, (uint32_t)kSliceThreads);
        uint32_t m = mine0;
        if (e0 != 0) {  // more than 512 entries (many staged batches, skewed data)
            __syncthreads();
            m = stage(e0, nit);
        }
        if (drains) {  // inclusive prefix of the run lengths over the chunk's entries
            const uint32_t inc = wave_incl_scan_dpp(m);
            if (lane == 63)
                sl.w_tot[wave] = inc;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int q = 0; q < kWavesS; q++)
                off += q < wave ? sl.w_tot[q] : 0u;
            sl.s_pin[tid] = off + inc;
        }
        __syncthreads();
        // a group = the kNI items j, j + kWavesS, ... of one wave.  Item run
        // parameters are wave-uniform and re-read from LDS where needed, so
        // nothing but the loaded dwords is live across a group's loads
        // (64 VGPRs: 32 waves per CU).  Issuing the next group's loads before
        // counting this one's measured slower.
        constexpr uint32_t kGrp = kNI * kWavesS;
        uint32_t ge = nit;  // entries [gs, ge): the current group
        auto run = [&](uint32_t jj, uint32_t& klo, uint32_t& khi) {
            const bool v = jj < ge;
            const uint32_t r = rfl(sl.s_run[v ? jj : 0u]);
            klo = v ? r & 0xffffu : 0u;
            khi = v ? r >> 16 : 0u;
        };
        // a buffer descriptor per item whose extent ends at the run's last
        // dword (so the loads need no per-lane bound); items start at
        // multiples of kPartChunk keys: dword-aligned
        auto issue = [&](uint32_t j, uint32_t p0, uint32_t (&w)[kNI][kKG]) -> uint32_t {
            uint32_t steps = 0;
#pragma unroll
            for (int q = 0; q < kNI; q++) {
                const uint32_t jj = j + q * kWavesS;
                uint32_t klo, khi;
                run(jj, klo, khi);
                const uint32_t jc = jj < ge ? jj : 0u;
                const uint32_t dlo = klo >> 1, dhi = (khi + 1) >> 1;
                const uint16_t* base = a.part2 + (uint64_t)rfl(sl.s_k[jc]) * a.part2_stride +
                                       (uint64_t)rfl(sl.s_base[jc]) * kPartChunk;
                const __amdgpu_buffer_rsrc_t src = uniform_rsrc(base, (uint64_t)dhi * 4u);
#pragma unroll
                for (int g = 0; g < kKG; g++)
                    w[q][g] = __builtin_amdgcn_raw_buffer_load_b32(src, (dlo + p0 + 64 * g + lane) * 4u, 0, 0);
                steps = max(steps, dhi - dlo);
            }
            return steps;
        };
        auto count = [&](uint32_t j, uint32_t p0, const uint32_t (&w)[kNI][kKG]) {
#pragma unroll
            for (int q = 0; q < kNI; q++) {
                uint32_t klo, khi;
                run(j + q * kWavesS, klo, khi);
                const uint32_t dlo = klo >> 1;
#pragma unroll
                for (int g = 0; g < kKG; g++) {
                    const uint32_t k0 = 2 * (dlo + p0 + 64 * g + lane);  // key index of the low half
                    // (part2 stores a key's low 16 bits: bits 14-15 are its slice's)
                    if (k0 >= klo && k0 < khi)
                        slice_count(h, w[q][g] & kSpanMask);
                    if (k0 + 1 >= klo && k0 + 1 < khi)
                        slice_count(h, (w[q][g] >> 16) & kSpanMask);
                }
            }
        };
        for (uint32_t gs = 0; gs < nit;) {
            if (drains) {  // the group: the longest run of entries whose events fit kDrainCap - since
                const uint32_t base = gs ? rfl(sl.s_pin[gs - 1]) : 0u, lim = kDrainCap - since;
                uint32_t lo = gs, hi = nit;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (rfl(sl.s_pin[mid]) - base > lim)
                        hi = mid;
                    else
                        lo = mid + 1;
                }
                ge = (lo == gs && since == 0) ? gs + 1 : lo;  // (a run never passes the cap alone)
                since += ge > gs ? rfl(sl.s_pin[ge - 1]) - base : 0u;
            }
            for (uint32_t j = gs + (uint32_t)wave; j < ge; j += kGrp) {
                uint32_t w[kNI][kKG];
                const uint32_t steps = issue(j, 0, w);
                count(j, 0, w);
                for (uint32_t p0 = 64 * kKG; p0 < steps; p0 += 64 * kKG) {  // runs longer than one pass (rare)
                    issue(j, p0, w);
                    count(j, p0, w);
                }
            }
            if (ge < nit) {  // the next run would pass the cap
                __syncthreads();
                drain();
                __syncthreads();
                since = 0;
            }
            gs = ge;
        }
    }
    __syncthreads();
    // low-byte plane: thread t owns bins [16t, +16) and [16(t + kSliceThreads), +16)
#pragma unroll
    for (int j = 0; j < kLoPer; j++) {
        const uint32_t b0 = 16u * (uint32_t)(tid + j * kSliceThreads);
        uint32_t incs[16];
        {
            const u32x4_t* hc = (const u32x4_t*)(h + b0 / 2);
            const u32x4_t c0 = hc[0], c1 = hc[1];
            const uint32_t w8[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
            for (int m = 0; m < 8; m++) {
                incs[2 * m] = w8[m] & 0xffffu;
                incs[2 * m + 1] = w8[m] >> 16;
            }
        }
        uint32_t words[4] = {l[j].x, l[j].y, l[j].z, l[j].w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t nw = 0;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const uint32_t nv = ((words[k] >> (8 * m)) & 0xffu) + incs[4 * k + m];
                nw |= (nv & 0xffu) << (8 * m);
                const uint32_t carry = nv & ~0xffu;
                if (carry)
                    a.hist[sb + b0 + 4 * k + m] += carry;  // u32 wrap, like the reference's atomic add
            }
            words[k] = nw;
        }
        lo4[tid + j * kSliceThreads] = u32x4_t{words[0], words[1], words[2], words[3]};
    }
}

__global__ void __launch_bounds__(kSliceThreads, 8) rx_slice_histo_kernel(HistoArgs a)  // 32 waves per CU
{
    __shared__ __attribute__((aligned(16))) uint32_t h[(kSliceSpan << kSliceBits) / 2];
    __shared__ SliceLds sl;
    slice_histo(a, blockIdx.x, h, sl);
}

}  // namespace dqdk
