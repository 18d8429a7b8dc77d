// emurx_parse.h — device-side restatement of the TRex-EMU receive path (gfx950).
//
// One frame per lane.  Byte sources (wave LDS slab or global memory), the RFC 1071 sum in
// dword form, ParsePacket / parsePacketL4 / processIpv6Options (src/emu/core/parser.go:
// 583-959) and the per-callback Namespace / Client rules of src/emu/plugins/* as device
// functions; the kernels that drive them are in emurx_kernels.hip.  The CPU oracle
// (oracle/emurx_oracle.c) is the line-by-line twin the parity tests compare with.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_tables.h"

namespace emurx {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
// LDS bytes staged per wave (64 frames).  7 KiB keeps a workgroup's LDS under 32 KiB, so
// five workgroups (20 waves) fit a CU; waves whose frames span more take the window path
// LDS staging slab per wave (emurx_kernels.hip): two sizes, chosen per launch (kStageNarrow
// gives 6 workgroups per CU instead of 5; waves wider than it take the window path)
constexpr uint32_t kStageWide = 7168, kStageNarrow = 6144;

// loads through the global address space (global_load_*): pointers rebuilt from integers or
// kept in a struct would otherwise compile to flat loads, which also count on lgkmcnt and
// make the compiler serialise them with LDS traffic
typedef unsigned emurx_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld16(const void* p) {
    const emurx_v4u v = *(const __attribute__((address_space(1))) emurx_v4u*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
typedef unsigned emurx_v3u __attribute__((ext_vector_type(3)));
__device__ __forceinline__ uint3 gld12(const void* p) {  // 4-byte aligned
    const emurx_v3u v = *(const __attribute__((address_space(1))) emurx_v3u*)p;
    return make_uint3(v.x, v.y, v.z);
}
__device__ __forceinline__ uint32_t gld4(const void* p) { return *(const __attribute__((address_space(1))) uint32_t*)p; }
__device__ __forceinline__ uint32_t gld1(const void* p) { return *(const __attribute__((address_space(1))) uint8_t*)p; }

// ---------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
// wave64 reductions on the DPP network (quad perms, row rotates, row broadcasts; result is
// read from lane 63 into a scalar register): no LDS traffic, 6 VALU + 1 readlane
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, kCtrl, kRowMask, 0xf, false);
}
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v, Op op) {
    v = op(v, dpp<0xb1>(v));        // quad_perm [1,0,3,2]
    v = op(v, dpp<0x4e>(v));        // quad_perm [2,3,0,1]
    v = op(v, dpp<0x124>(v));       // row_ror:4
    v = op(v, dpp<0x128>(v));       // row_ror:8
    v = op(v, dpp<0x142, 0xa>(v));  // row_bcast:15
    v = op(v, dpp<0x143, 0xc>(v));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return wave_reduce(v, [](uint32_t x, uint32_t y) { return min(x, y); });
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_reduce(v, [](uint32_t x, uint32_t y) { return max(x, y); });
}
// Namespace-owner packing (emurx_route.hip, k_rx kind 2): the offset of `tile` in each owner's
// region = its group's offset (grp_off, k_route_scan) + the counts of the group's earlier
// tiles (tile_cnt[t][owner], 64 tiles per group).  Called by one whole wave; lane 0 writes
// s_toff[0 .. parts).
// The loads of tile_offsets alone (x, y: the counts of the group's earlier tiles, lane l's
// tile; g: lane l's group offset for owner l), so that a kernel can issue them ahead of a
// wait it makes anyway (k_rx<2>: before its staging wait) and finish with tile_offsets_sum.
struct TileOffLoads {
    uint4 x, y;
    uint32_t g;
};
__device__ __forceinline__ TileOffLoads tile_offsets_issue(const uint32_t* tile_cnt, const uint32_t* grp_off,
                                                           uint32_t parts, uint32_t tile, uint32_t lane) {
    TileOffLoads t{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), 0u};
    const uint32_t g0 = tile & ~63u;
    if (g0 + lane < tile) {
        const uint4* q = reinterpret_cast<const uint4*>(tile_cnt + (size_t)(g0 + lane) * 16);
        t.x = q[0];
        t.y = q[1];
    }
    if (lane < parts) t.g = grp_off[(tile / 64) * 16 + lane];
    return t;
}
template <class R>
__device__ __forceinline__ void tile_offsets_sum(const TileOffLoads& t, uint32_t parts, uint32_t lane, uint32_t* s_toff,
                                                 R reduce_sum) {
    const uint32_t c[EMURX_MAX_PARTS] = {t.x.x, t.x.y, t.x.z, t.x.w, t.y.x, t.y.y, t.y.z, t.y.w};
#pragma unroll
    for (uint32_t k = 0; k < EMURX_MAX_PARTS; ++k) {
        if (k >= parts) break;
        const uint32_t sum = reduce_sum(c[k]);
        const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)t.g, (int)k);
        if (lane == 0) s_toff[k] = g + sum;
    }
}
template <class R>
__device__ __forceinline__ void tile_offsets(const uint32_t* tile_cnt, const uint32_t* grp_off, uint32_t parts,
                                             uint32_t tile, uint32_t lane, uint32_t* s_toff, R reduce_sum) {
    const uint32_t g0 = tile & ~63u;
    uint4 x = make_uint4(0, 0, 0, 0), y = x;
    if (g0 + lane < tile) {
        const uint4* q = reinterpret_cast<const uint4*>(tile_cnt + (size_t)(g0 + lane) * 16);
        x = q[0];
        y = q[1];
    }
    const uint32_t c[EMURX_MAX_PARTS] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
    for (uint32_t k = 0; k < EMURX_MAX_PARTS; ++k) {
        if (k >= parts) break;
        const uint32_t sum = reduce_sum(c[k]);
        if (lane == 0) s_toff[k] = grp_off[(tile / 64) * 16 + k] + sum;
    }
}

// The CTunnelKey VLAN words ParsePacket leaves for a frame (parser.go:801-818), from its
// length and bytes 12..19 alone: tag 0 when bytes 12..13 are 0x8100 / 0x88a8 and the frame
// holds it, tag 1 likewise after it unless PPPoE follows tag 0.  parse_flat and parse_packet
// set r.vlan0 / r.vlan1 to exactly these (the owner-count pass routes by them).
__device__ __forceinline__ void l2_vlans(uint32_t len, uint32_t w12, uint32_t w16, uint32_t& v0, uint32_t& v1) {
    const uint32_t e0 = w12 >> 16, e1 = w16 >> 16;  // big-endian words of bytes 12..15, 16..19
    const bool g0 = len >= 18 && (e0 == 0x8100 || e0 == 0x88A8);
    const bool g1 = g0 && len >= 22 && (e1 == 0x8100 || e1 == 0x88A8);
    v0 = g0 ? (w12 & 0xffff0fffu) : 0u;
    v1 = g1 ? (w16 & 0xffff0fffu) : 0u;
}

// lanes below this one in mask m
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---------------------------------------------------------------------------------------
// RFC 1071 sum, restated for dword loads.
// Go (layers/tcpip.go:76-94) adds big-endian byte pairs of the span into a uint32 and
// folds; the span is valid iff the folded value is 0xffff.  Modulo 0xffff, 2^16 == 1 and
// 256*256 == 1, so a little-endian dword at an aligned address contributes each byte with
// weight 256^(address & 1).  Summing masked aligned dwords therefore gives
//   S_go == T * 256^(1 - (span_start & 1))   (mod 0xffff)
// and S_go + pseudo == 0 (mod 0xffff) with a non-zero total <=> Go's check passes.
// ---------------------------------------------------------------------------------------
// v_sad_u16(w, 0, acc) = acc + (w & 0xffff) + (w >> 16): one VALU per dword, and
// == sum of w (mod 0xffff) because 2^16 == 1.  Zero iff every masked byte is zero.
__device__ __forceinline__ uint32_t sad16(uint32_t w, uint32_t acc) { return __builtin_amdgcn_sad_u16(w, 0u, acc); }
__device__ __forceinline__ uint32_t fold16(uint32_t x) {
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return x;  // <= 0xffff, == x mod 0xffff (0xffff stands for 0)
}
// the sum of the span's big-endian 16-bit words (mod 0xffff) from its aligned-dword sum T
__device__ __forceinline__ uint32_t be_domain(uint32_t T, uint32_t a_start) {
    uint32_t t = fold16(T);
    return (a_start & 1u) ? t : (((t << 8) | (t >> 8)) & 0xffffu);
}
// tcpipChecksum(span, pcs) == 0  <=>  pcs + S == 0 (mod 0xffff) and the u32 sum is non-zero
__device__ __forceinline__ bool csum_ok(uint32_t T, uint32_t a_start, uint32_t pcs) {
    uint32_t x = fold16(be_domain(T, a_start) + pcs);
    return (x == 0xffffu || x == 0u) && !(T == 0 && pcs == 0);
}
// sum over the bytes [a, a + n) of a dword sequence w[k] (byte a at dword a >> 2):
// head / body / tail masks, body unmasked
#ifndef EMURX_SHORTSUM
#define EMURX_SHORTSUM 0
#endif
template <class A>
__device__ __forceinline__ uint32_t dword_sum(const A& w, uint32_t a, uint32_t n) {
    if (n == 0) return 0;
    const uint32_t e = a + n, k0 = a >> 2, k1 = (e - 1) >> 2;
    const uint32_t hm = 0xffffffffu << (8 * (a & 3));
    const uint32_t tm = 0xffffffffu >> (8 * ((0u - e) & 3));
#if EMURX_SHORTSUM
    // a span of at most 64 bytes (17 dwords): every dword read at once, the ones past the span
    // masked to nothing (one LDS round trip instead of one per four dwords); wave-uniform test
    if (__builtin_amdgcn_ballot_w64(k1 - k0 > 16) == 0) {
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t j = 0; j <= 16; ++j) {
            const uint32_t k = k0 + j;
            const uint32_t m = k > k1 ? 0u : (j == 0 ? hm : 0xffffffffu) & (k == k1 ? tm : 0xffffffffu);
            acc = sad16(w[k] & m, acc);  // read unconditionally: a dword past the span is in LDS
        }
        return acc;
    }
#endif
    const uint32_t w0 = w[k0] & hm;
    if (k0 == k1) return sad16(w0 & tm, 0);
    uint32_t acc = sad16(w0, 0), k = k0 + 1;
    for (; k + 4 <= k1; k += 4) {
        const uint32_t x0 = w[k], x1 = w[k + 1], x2 = w[k + 2], x3 = w[k + 3];
        acc = sad16(x3, sad16(x2, sad16(x1, sad16(x0, acc))));
    }
    for (; k < k1; ++k) acc = sad16(w[k], acc);
    return sad16(w[k1] & tm, acc);
}
// the same over a fixed length N (a multiple of 4) from byte a: N/4 + 1 dwords, straight-line
// (the last one masked to nothing when a is dword-aligned; reading it is harmless in LDS)
template <uint32_t N, class A>
__device__ __forceinline__ uint32_t dword_sum_fixed(const A& w, uint32_t a) {
    static_assert(N % 4 == 0 && N >= 4, "whole dwords");
    const uint32_t k0 = a >> 2, sh = 8 * (a & 3);
    const uint32_t hm = 0xffffffffu << sh;
    uint32_t acc = sad16(w[k0] & hm, 0);
#pragma unroll
    for (uint32_t j = 1; j < N / 4; ++j) acc = sad16(w[k0 + j], acc);
    return sad16(w[k0 + N / 4] & ~hm, acc);
}
// bytes [lo, hi) of a 16-byte vector (indices may fall outside 0..16)
__device__ __forceinline__ uint32_t keep(int lo, int hi, int d) {
    const int a = lo - 4 * d, b = hi - 4 * d;
    const uint32_t m1 = a <= 0 ? 0xffffffffu : (a >= 4 ? 0u : (0xffffffffu << (8 * a)));
    const uint32_t m2 = b >= 4 ? 0xffffffffu : (b <= 0 ? 0u : (0xffffffffu >> (8 * (4 - b))));
    return m1 & m2;
}
__device__ __forceinline__ uint32_t sad_vec(const uint4& x, uint32_t acc) {
    return sad16(x.w, sad16(x.z, sad16(x.y, sad16(x.x, acc))));
}
__device__ __forceinline__ uint32_t sad_vec_masked(const uint4& x, int lo, int hi, uint32_t acc) {
    return sad16(x.w & keep(lo, hi, 3), sad16(x.z & keep(lo, hi, 2),
                 sad16(x.y & keep(lo, hi, 1), sad16(x.x & keep(lo, hi, 0), acc))));
}
// the same sum over global bytes p[0, n) with 16-byte loads, four in flight per step
__device__ __forceinline__ uint32_t glb_sum(const uint8_t* p, uint32_t n) {
    if (n == 0) return 0;
    const uintptr_t a = (uintptr_t)p, e = a + n;
    const uint8_t* v = reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)15);
    const uint32_t nv = (uint32_t)((((e + 15) & ~(uintptr_t)15) - (a & ~(uintptr_t)15)) >> 4);
    const int h = (int)(a & 15), t = 16 - (int)((0u - (uint32_t)e) & 15);  // keep [h, 16) / [0, t)
    if (nv == 1) return sad_vec_masked(gld16(v), h, t, 0);
    uint32_t acc = sad_vec_masked(gld16(v), h, 16, 0), k = 1;
    for (; k + 4 <= nv - 1; k += 4) {
        const uint4 x0 = gld16(v + 16 * k), x1 = gld16(v + 16 * (k + 1)), x2 = gld16(v + 16 * (k + 2)),
                    x3 = gld16(v + 16 * (k + 3));
        acc = sad_vec(x3, sad_vec(x2, sad_vec(x1, sad_vec(x0, acc))));
    }
    for (; k < nv - 1; ++k) acc = sad_vec(gld16(v + 16 * k), acc);
    return sad_vec_masked(gld16(v + 16 * (nv - 1)), 0, t, acc);
}

// ---------------------------------------------------------------------------------------
// byte sources.  LdsSrc: the wave's contiguous LDS copy of its frames (fast path).
// WinSrc: waves whose frames do not fit the slab (IMIX, jumbo) — each lane holds a 128-byte
// window of its own frame in LDS (headers), everything past it is read from global memory
// (the checksum spans, with 16-byte loads).
// ---------------------------------------------------------------------------------------
struct LdsSrc {
    const uint8_t* b8;    // block LDS
    const uint32_t* b32;  // same array, dword view
    uint32_t base;        // LDS byte index of frame byte 0 (== global address mod 16)
    __device__ __forceinline__ uint32_t u8(uint32_t i) const { return b8[base + i]; }
    __device__ __forceinline__ uint32_t sum(uint32_t s, uint32_t n) const { return dword_sum(b32, base + s, n); }
    template <uint32_t N>
    __device__ __forceinline__ uint32_t sum_fixed(uint32_t s) const { return dword_sum_fixed<N>(b32, base + s); }
    __device__ __forceinline__ uint32_t at(uint32_t s) const { return base + s; }
};
// window layout: vector k of lane l at wave slab byte k * 1024 + l * 16 (LDS-DMA order)
struct WinDw {
    const uint32_t* p;  // slab dword of lane l's vector 0
    __device__ __forceinline__ uint32_t operator[](uint32_t j) const { return p[((j >> 2) << 8) + (j & 3)]; }
};
struct WinSrc {
    const uint8_t* b8;
    const uint32_t* b32;
    uint32_t wbase;     // LDS byte index of this lane's vector 0
    uint32_t head;      // frame byte 0 within vector 0 (== global address mod 16)
    uint32_t wlim;      // frame bytes [0, wlim) are in the window
    const uint8_t* f;   // frame byte 0 (global)
    __device__ __forceinline__ uint32_t u8(uint32_t i) const {
        if (i < wlim) {
            const uint32_t b = head + i;
            return b8[wbase + ((b >> 4) << 10) + (b & 15)];
        }
        return gld1(f + i);
    }
    __device__ __forceinline__ uint32_t sum(uint32_t s, uint32_t n) const {
        const uint32_t e = s + n, m = min(e, wlim);
        uint32_t acc = 0;
        if (s < m) acc = dword_sum(WinDw{b32 + (wbase >> 2)}, head + s, m - s);
        const uint32_t g = max(s, wlim);
        if (e > g) acc += glb_sum(f + g, e - g);
        return acc;
    }
    // fixed length N inside the window: straight-line (dword N/4 + 1 still lies in it)
    template <uint32_t N>
    __device__ __forceinline__ uint32_t sum_fixed(uint32_t s) const {
        return s + N <= wlim ? dword_sum_fixed<N>(WinDw{b32 + (wbase >> 2)}, head + s) : sum(s, N);
    }
    __device__ __forceinline__ uint32_t at(uint32_t s) const { return (uint32_t)(uintptr_t)(f + s); }
};
// tcpipChecksum(p[s:s+n], pcs) == 0
template <class S>
__device__ __forceinline__ bool csum(const S& src, uint32_t s, uint32_t n, uint32_t pcs) {
    return csum_ok(src.sum(s, n), src.at(s), pcs);
}
// sum of the big-endian 16-bit words of p[s:s+n] (n even), mod 0xffff: GetPhCs's address part
template <class S>
__device__ __forceinline__ uint32_t pseudo(const S& src, uint32_t s, uint32_t n) {
    return be_domain(src.sum(s, n), src.at(s));
}

template <class S>
__device__ __forceinline__ uint32_t be16(const S& s, uint32_t i) { return (s.u8(i) << 8) | s.u8(i + 1); }
template <class S>
__device__ __forceinline__ uint32_t be32(const S& s, uint32_t i) {
    return (s.u8(i) << 24) | (s.u8(i + 1) << 16) | (s.u8(i + 2) << 8) | s.u8(i + 3);
}
template <class S>  // bytes i..i+3 as a little-endian word (the table key encoding)
__device__ __forceinline__ uint32_t le32(const S& s, uint32_t i) {
    return s.u8(i) | (s.u8(i + 1) << 8) | (s.u8(i + 2) << 16) | (s.u8(i + 3) << 24);
}
// Staged frames: 32-bit fields from the two aligned LDS dwords that hold them (v_alignbyte)
// instead of four byte reads (measured C -3 %, D -1.6 %, B -2 %); the second dword may lie
// past the frame, harmless in LDS and masked out by the shift when the field is aligned
__device__ __forceinline__ uint32_t le32(const LdsSrc& s, uint32_t i) {
    const uint32_t a = s.base + i, k = a >> 2;
    return __builtin_amdgcn_alignbyte(s.b32[k + 1], s.b32[k], a & 3);
}
__device__ __forceinline__ uint32_t be32(const LdsSrc& s, uint32_t i) { return __builtin_bswap32(le32(s, i)); }
// ---------------------------------------------------------------------------------------
// parse state == ParserPacketState + CTunnelData + outcome
// ---------------------------------------------------------------------------------------
struct Rec {
    uint32_t ns, cl, vlan0, vlan1;
    uint32_t vport, l3, l4, l7, l7len;
    uint32_t nh, proto, status, flags;
    // L4 checksum deferred to the wave-cooperative pass (WinSrc spans past the window):
    // bytes [dstart, dstart + dlen) with pseudo sum dpcs; on failure the outcome becomes dfail
    uint32_t dstart, dlen, dpcs, dfail;
    uint32_t flow;  // EMURX_FLOW_* / flow id (transport handler decision)
};

__device__ __forceinline__ void invoke(Rec& r, uint32_t cb, uint32_t cb_mask) {
    r.proto = cb;
    if (cb_mask & (1u << cb)) r.status = EMURX_ST_OK;
    else if (cb == EMURX_CB_EAPOL) r.status = EMURX_ST_PANIC_NIL_EAPOL;  // nil ParserCb :789
    else r.status = EMURX_ST_NOT_SUPPORTED;                              // parserNotSupported
}
__device__ __forceinline__ void fail(Rec& r, uint32_t st) { r.status = st; r.proto = EMURX_CB_NONE; }

__device__ __forceinline__ bool span_ok(uint32_t l4, uint32_t l4len) {
    return ((l4 + l4len) & 0xffffu) >= l4;  // Go slice p[L4:L4+l4len] with uint16 end
}

// the L4 checksum of parsePacketL4.  LdsSrc: now.  WinSrc: now when the span lies in the
// lane's window, else deferred to coop_checksum_rows() (the caller proceeds as if it passed; the
// cooperative pass applies `fail_st` afterwards, see settle_deferred)
template <class S>
__device__ __forceinline__ bool csum_l4(const S& s, Rec& r, uint32_t at, uint32_t n, uint32_t pcs, uint32_t fail_st) {
    return csum(s, at, n, pcs);
}
// EMURX_WSKIP (default since round 4; =0 the round-3 re-read): the span's bytes inside the window are summed from LDS
// here and folded into the deferred pseudo sum (the byte-pair sum is linear mod 0xffff, and
// be_domain with the span's own start parity orients both parts alike), so the cooperative
// pass reads only the bytes past the window: every span byte crosses HBM once
#ifndef EMURX_WSKIP
#define EMURX_WSKIP 1
#endif
template <>
__device__ __forceinline__ bool csum_l4<WinSrc>(const WinSrc& s, Rec& r, uint32_t at, uint32_t n, uint32_t pcs,
                                                uint32_t fail_st) {
    if (at + n <= s.wlim || n == 0) return csum(s, at, n, pcs);
    uint32_t st = at, pw = pcs;
    if (EMURX_WSKIP && at < s.wlim) {
        const uint32_t tw = dword_sum(WinDw{s.b32 + (s.wbase >> 2)}, s.head + at, s.wlim - at);
        pw = pcs + be_domain(tw, s.at(at));  // tw == 0 leaves pcs as it was (Go's all-zero case)
        st = s.wlim;
    }
    r.dstart = st;
    r.dlen = at + n - st;
    r.dpcs = pw;
    r.dfail = fail_st | ((s.at(at) & 1u) << 16);  // the span's start parity (csum_ok's a_start)
    return true;
}

// processIpv6Options parser.go:726-746; false on Go's out-of-range p[i+1]
template <class S>
__device__ bool ipv6_options(const S& s, uint32_t p0, int size, uint32_t& flags) {
    int i = 0;
    uint32_t nh = s.u8(p0);
    for (;;) {
        if (nh == 0) {
            i++;
        } else if (nh == 5) {
            flags |= EMURX_FLAG_RTALERT;
            return true;
        } else {
            if (i + 1 >= size) return false;
            i = i + 2 + (int)s.u8(p0 + i + 1);
        }
        if (i > size - 1) return true;
        nh = s.u8(p0 + i);
    }
}

// Parser.parsePacketL4 parser.go:583-724
template <class S>
__device__ __forceinline__ void parse_l4(const S& s, uint32_t len, Rec& r, uint32_t nextHdr, uint32_t pcs,
                         uint32_t l4len, bool v6, uint32_t cb_mask) {
    r.nh = nextHdr;
    const uint32_t L4 = r.l4;
    switch (nextHdr) {
    case 1:  // ICMPv4
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!csum_l4(s, r, L4, l4len, 0, EMURX_ST_ICMPV4_CS)) { fail(r, EMURX_ST_ICMPV4_CS); return; }
        r.l7 = (L4 + 8) & 0xffff;
        invoke(r, EMURX_CB_ICMP, cb_mask);
        return;
    case 2:  // IGMP (no checksum in the parser)
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        invoke(r, EMURX_CB_IGMP, cb_mask);
        return;
    case 6: {  // TCP
        if (l4len < 20) { fail(r, EMURX_ST_TCP_TOO_SHORT); return; }
        if (((L4 + 12) & 0xffff) >= len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        uint32_t tcplen = (s.u8((L4 + 12) & 0xffff) >> 4) << 2;
        if (l4len < tcplen) { fail(r, EMURX_ST_TCP_TOO_SHORT); return; }
        r.l7 = (L4 + tcplen) & 0xffff;
        r.l7len = (l4len - tcplen) & 0xffff;
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!csum_l4(s, r, L4, l4len, pcs, EMURX_ST_TCP_CS)) { fail(r, EMURX_ST_TCP_CS); return; }
        invoke(r, EMURX_CB_TCP, cb_mask);
        return;
    }
    case 17: {  // UDP
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_UDP_TOO_SHORT); return; }
        r.l7len = (l4len - 8) & 0xffff;
        if (be16(s, L4 + 6) > 0) {
            if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
            if (!csum_l4(s, r, L4, l4len, pcs, EMURX_ST_UDP_CS)) { fail(r, EMURX_ST_UDP_CS); return; }
        }
        r.l7 = (L4 + 8) & 0xffff;
        uint32_t src = be16(s, L4), dst = be16(s, L4 + 2);
        uint32_t cb = EMURX_CB_UDP;
        if (dst == 5353) cb = EMURX_CB_MDNS;
        else if (v6) { if (src == 547 && dst == 546) cb = EMURX_CB_DHCPV6; }
        else if (src == 67 && dst == 68) cb = EMURX_CB_DHCP;
        else if (dst == 67 && (src == 67 || src == 68)) cb = EMURX_CB_DHCPSRV;
        invoke(r, cb, cb_mask);
        return;
    }
    case 58: {  // ICMPv6
        if (len < ((L4 + 4) & 0xffff)) { fail(r, EMURX_ST_ICMPV6_TOO_SHORT); return; }
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!csum_l4(s, r, L4, l4len, pcs, EMURX_ST_ICMPV6_CS)) { fail(r, EMURX_ST_ICMPV6_CS); return; }
        uint32_t t = s.u8(L4);
        bool okt = (t >= 1 && t <= 4) || (t >= 128 && t <= 136);
        if (okt) invoke(r, EMURX_CB_ICMPV6, cb_mask);
        else fail(r, EMURX_ST_ICMPV6_UNSUPPORTED);
        return;
    }
    default:
        fail(r, EMURX_ST_L4_UNSUPPORTED);
        return;
    }
}

// pseudo-header partial sums (IPv4Header.GetPhCs ip4.go:49-58, IPv6Header.GetPhCs
// ip6.go:126-134) are taken mod 0xffff: the checksum verdict depends on the sum only mod
// 0xffff, and with the protocol term (never 0 where a pseudo header is used) never zero.
// Parser.ParsePacket parser.go:756-959
template <class S>
__device__ __forceinline__ void parse_packet(const S& s, uint32_t len, uint32_t vport, uint32_t cb_mask, Rec& r) {
    r.ns = EMURX_ID_NONE; r.cl = EMURX_ID_NONE;
    r.vlan0 = 0; r.vlan1 = 0; r.vport = vport;
    r.l3 = r.l4 = r.l7 = r.l7len = 0;
    r.nh = 0; r.proto = EMURX_CB_NONE; r.status = EMURX_ST_OK; r.flags = 0;
    r.dlen = 0;
    r.flow = EMURX_FLOW_NONE;
    if (len < 14) { fail(r, EMURX_ST_PACKET_TOO_SHORT); return; }
    uint32_t offset = 14;
    uint32_t nextHdr = be16(s, 12);
    int vlanIndex = 0;
    uint32_t l4 = 0, l4len = 0, nh = 0, pcs = 0;  // the L4 tail's inputs
    bool v6 = false;
    for (;;) {
        if (nextHdr == 0x8100 || nextHdr == 0x88A8) {
            if (len < offset + 4) { fail(r, EMURX_ST_DOT1Q_TOO_SHORT); return; }
            if (vlanIndex > 1) { fail(r, EMURX_ST_TOO_MANY_DOT1Q); return; }
            uint32_t val = be32(s, offset - 2) & 0xffff0fffu;
            if (vlanIndex == 0) r.vlan0 = val; else r.vlan1 = val;
            vlanIndex++;
            nextHdr = be16(s, offset + 2);
            if (nextHdr == 0x8863 || nextHdr == 0x8864) { invoke(r, EMURX_CB_PPP, cb_mask); return; }
            offset += 4;
            continue;
        }
        if (nextHdr == 0x0800) {  // IPv4
            r.l3 = offset;
            if (len < offset + 20) { fail(r, EMURX_ST_IPV4_TOO_SHORT); return; }
            uint32_t b0 = s.u8(offset);
            if ((b0 >> 4) != 4) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint32_t frag = be16(s, offset + 6);
            if ((frag & 0x1fff) != 0 || (frag & 0x2000) != 0) { fail(r, EMURX_ST_IPV4_FRAGMENT); return; }
            uint32_t hdr = (b0 & 0xf) << 2;
            if (hdr < 20) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            if (len < offset + hdr) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint32_t totlen = be16(s, offset + 2);
            if (len < ((offset + totlen) & 0xffff)) { fail(r, EMURX_ST_IPV4_TOO_SHORT); return; }
            const uint32_t th = hdr == 20 ? s.template sum_fixed<20>(offset) : s.sum(offset, hdr);
            if (!csum_ok(th, s.at(offset), 0)) { fail(r, EMURX_ST_IPV4_CS); return; }
            l4len = (totlen - hdr) & 0xffff;
            l4 = offset + hdr;
            nh = s.u8(offset + 9);
            pcs = be_domain(s.template sum_fixed<8>(offset + 12), s.at(offset + 12)) + nh + l4len;  // src, dst, 0|proto, len
            break;
        }
        if (nextHdr == 0x86DD) {  // IPv6
            r.l3 = offset;
            if (len < offset + 40) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if ((s.u8(offset) >> 4) != 6) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            uint32_t plen = be16(s, offset + 4);
            if (len < ((offset + 40 + plen) & 0xffff)) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if (s.u8(offset + 7) == 0) { fail(r, EMURX_ST_IPV6_HOPLIMIT); return; }
            uint32_t osize = 0;
            l4 = offset + 40;
            l4len = plen;
            nh = s.u8(offset + 6);
            for (;;) {
                bool ext = nh == 0 || nh == 60 || nh == 43 || nh == 51 || nh == 50 || nh == 135 ||
                           nh == 139 || nh == 140;
                if (!ext) break;
                if (l4len < 8) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
                if (l4 + 2 > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
                uint32_t hl = (s.u8(l4 + 1) << 3) + 8;
                if (l4len < hl) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
                if (l4 + hl > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
                uint32_t nnh = s.u8(l4);
                if (!ipv6_options(s, l4 + 2, (int)hl - 2, r.flags)) { fail(r, EMURX_ST_PANIC_IPV6_OPT); return; }
                nh = nnh;
                l4len -= hl;
                osize += hl;
                l4 += hl;
            }
            if (nh == 44) { fail(r, EMURX_ST_IPV6_FRAGMENT); return; }
            if (nh == 194) { fail(r, EMURX_ST_IPV6_JUMBO); return; }
            if (nh == 59) { fail(r, EMURX_ST_IPV6_EMPTY); return; }
            v6 = true;
            pcs = be_domain(s.template sum_fixed<32>(offset + 8), s.at(offset + 8)) + ((plen - osize) & 0xffff) + nh;  // src, dst, len, 0|nh
            break;
        }
        if (nextHdr == 0x888E) {  // EAPOL
            if (len < offset + 4) { fail(r, EMURX_ST_EAPOL_TOO_SHORT); return; }
            r.l3 = offset;
            invoke(r, EMURX_CB_EAPOL, cb_mask);
            return;
        }
        if (nextHdr == 0x0806) {  // ARP, ARPHeaderSize 28
            if (len < offset + 28) { fail(r, EMURX_ST_ARP_TOO_SHORT); return; }
            r.l3 = offset;
            invoke(r, EMURX_CB_ARP, cb_mask);
            return;
        }
        if (nextHdr == 0x8863 || nextHdr == 0x8864) { invoke(r, EMURX_CB_PPP, cb_mask); return; }
        fail(r, EMURX_ST_L3_UNSUPPORTED);
        return;
    }
    // IPv4 / IPv6: one parsePacketL4 for the wave
    r.l4 = l4;
    parse_l4(s, len, r, nh, pcs, l4len, v6, cb_mask);
}

// ---------------------------------------------------------------------------------------
// The same ParsePacket, written for the staged (LDS) path with as little divergent control
// flow as the Go semantics allow: every check of a layer is evaluated and the first failing
// one (in Go's order) is picked by selects, every checksum of a frame is one dword-sum call
// whose length is zero where Go would not reach it.  Reads past a frame stay inside the
// workgroup's LDS (out-of-range LDS reads return 0 on CDNA), so evaluating a check Go would
// not reach is harmless; only the loop bounds (checksum spans, IPv6 extension headers) must
// be the ones Go would use.  Field values on every return path equal parse_packet's.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void first(uint32_t& st, bool cond, uint32_t code) {
    st = (st == EMURX_ST_OK && cond) ? code : st;
}

// EMURX_DWFIELDS: header fields of the staged path extracted from aligned-dword words (v_alignbyte)
// instead of byte reads (A/B)
#ifndef EMURX_DWFIELDS
#define EMURX_DWFIELDS 0
#endif
// Parser.parsePacketL4 parser.go:583-724, flat
__device__ __forceinline__ void parse_l4_flat(const LdsSrc& s, uint32_t len, Rec& r, uint32_t nextHdr, uint32_t pcs,
                                              uint32_t l4len, bool v6, uint32_t cb_mask) {
    r.nh = nextHdr;
    const uint32_t L4 = r.l4;
    const bool p1 = nextHdr == 1, p2 = nextHdr == 2, p6 = nextHdr == 6, p17 = nextHdr == 17, p58 = nextHdr == 58;
    const uint32_t L4_8 = (L4 + 8) & 0xffff, L4_4 = (L4 + 4) & 0xffff, L4_12 = (L4 + 12) & 0xffff;
    const bool sok = span_ok(L4, l4len);
#if EMURX_DWFIELDS
    // the L4 header's fields from three aligned-dword words (bytes L4..L4+7, L4+12..L4+15)
    // instead of eight byte reads; a staged frame's L4 + 12 never wraps the uint16
    const uint32_t P0 = le32(s, L4), P4 = le32(s, L4 + 4), P12 = le32(s, L4 + 12);
    const uint32_t tcplen = ((P12 & 0xff) >> 4) << 2;
    const bool ucs = (P4 >> 16) != 0;  // UDP checksum present (bytes L4+6, L4+7)
#else
    const uint32_t tcplen = (s.u8(L4_12) >> 4) << 2;
    const bool ucs = be16(s, L4 + 6) > 0;  // UDP checksum present
#endif
    uint32_t st = EMURX_ST_OK;
    bool tcp_hdr = false;  // TCP got past its length checks (L7 / L7Len are set)
    if (p1) {
        first(st, len < L4_8, EMURX_ST_ICMPV4_TOO_SHORT);
        first(st, !sok, EMURX_ST_PANIC_L4LEN);
    } else if (p2) {
        first(st, len < L4_8, EMURX_ST_ICMPV4_TOO_SHORT);
    } else if (p6) {
        first(st, l4len < 20, EMURX_ST_TCP_TOO_SHORT);
        first(st, L4_12 >= len, EMURX_ST_PANIC_L4LEN);
        first(st, l4len < tcplen, EMURX_ST_TCP_TOO_SHORT);
        tcp_hdr = st == EMURX_ST_OK;
        first(st, !sok, EMURX_ST_PANIC_L4LEN);
    } else if (p17) {
        first(st, len < L4_8, EMURX_ST_UDP_TOO_SHORT);
        first(st, ucs && !sok, EMURX_ST_PANIC_L4LEN);
    } else if (p58) {
        first(st, len < L4_4, EMURX_ST_ICMPV6_TOO_SHORT);
        first(st, !sok, EMURX_ST_PANIC_L4LEN);
    } else {
        st = EMURX_ST_L4_UNSUPPORTED;
    }
    const bool need = st == EMURX_ST_OK && (p1 || p6 || p58 || (p17 && ucs));
    const bool cs_ok = csum(s, L4, need ? l4len : 0u, p1 ? 0u : pcs);
    first(st, need && !cs_ok, p1 ? EMURX_ST_ICMPV4_CS : p6 ? EMURX_ST_TCP_CS : p17 ? EMURX_ST_UDP_CS : EMURX_ST_ICMPV6_CS);
    // L7 / L7Len as Go leaves them on each path (set before the checksum for TCP, L7Len
    // before it for UDP, L7 only on success for ICMP and UDP)
    r.l7len = tcp_hdr ? ((l4len - tcplen) & 0xffff) : (p17 && len >= L4_8) ? ((l4len - 8) & 0xffff) : 0u;
    r.l7 = tcp_hdr ? ((L4 + tcplen) & 0xffff) : ((p1 || p17) && st == EMURX_ST_OK) ? L4_8 : 0u;
#if EMURX_DWFIELDS
    const uint32_t src = ((P0 & 0xff) << 8) | ((P0 >> 8) & 0xff), dst = (((P0 >> 16) & 0xff) << 8) | (P0 >> 24),
                   t6 = P0 & 0xff;
#else
    const uint32_t src = be16(s, L4), dst = be16(s, L4 + 2), t6 = s.u8(L4);
#endif
    uint32_t cb = p1 ? EMURX_CB_ICMP : p2 ? EMURX_CB_IGMP : p6 ? EMURX_CB_TCP : p58 ? EMURX_CB_ICMPV6 : EMURX_CB_UDP;
    if (p17) {
        cb = dst == 5353 ? EMURX_CB_MDNS
           : v6 ? ((src == 547 && dst == 546) ? EMURX_CB_DHCPV6 : EMURX_CB_UDP)
           : (src == 67 && dst == 68) ? EMURX_CB_DHCP
           : (dst == 67 && (src == 67 || src == 68)) ? EMURX_CB_DHCPSRV : EMURX_CB_UDP;
    }
    first(st, p58 && !((t6 >= 1 && t6 <= 4) || (t6 >= 128 && t6 <= 136)), EMURX_ST_ICMPV6_UNSUPPORTED);
    if (st == EMURX_ST_OK) invoke(r, cb, cb_mask);
    else fail(r, st);
}

// Parser.ParsePacket parser.go:756-959, flat (staged frames)
__device__ __forceinline__ void parse_flat(const LdsSrc& s, uint32_t len, uint32_t vport, uint32_t cb_mask, Rec& r) {
    r.ns = EMURX_ID_NONE; r.cl = EMURX_ID_NONE;
    r.vlan0 = 0; r.vlan1 = 0; r.vport = vport;
    r.l3 = r.l4 = r.l7 = r.l7len = 0;
    r.nh = 0; r.proto = EMURX_CB_NONE; r.status = EMURX_ST_OK; r.flags = 0;
    r.dlen = 0;
    r.flow = EMURX_FLOW_NONE;
    // ---- L2: at most two tags, a third is errToManyDot1q; PPPoE right after a tag ----
    auto is_tag = [](uint32_t x) { return x == 0x8100 || x == 0x88A8; };
    auto is_ppp = [](uint32_t x) { return x == 0x8863 || x == 0x8864; };
    uint32_t st = EMURX_ST_OK;
    first(st, len < 14, EMURX_ST_PACKET_TOO_SHORT);
#if EMURX_DWFIELDS
    // bytes 12..23 as three big-endian words from four aligned dwords (the EtherType / TPID
    // words and the CTunnelKey VLAN words) instead of six byte reads and two word reads
    const uint32_t W12 = be32(s, 12), W16 = be32(s, 16), W20 = be32(s, 20);
    const uint32_t e0 = W12 >> 16, e1 = W16 >> 16, e2 = W20 >> 16;
#else
    const uint32_t e0 = be16(s, 12), e1 = be16(s, 16), e2 = be16(s, 20);
#endif
    const bool t0 = st == EMURX_ST_OK && is_tag(e0);
    first(st, t0 && len < 18, EMURX_ST_DOT1Q_TOO_SHORT);
    const bool g0 = t0 && st == EMURX_ST_OK;  // tag 0 parsed
    const bool ppp0 = g0 && is_ppp(e1);
    const bool t1 = g0 && !ppp0 && is_tag(e1);
    first(st, t1 && len < 22, EMURX_ST_DOT1Q_TOO_SHORT);
    const bool g1 = t1 && st == EMURX_ST_OK;
    const bool ppp1 = g1 && is_ppp(e2);
    const bool t2 = g1 && !ppp1 && is_tag(e2);
    first(st, t2 && len < 26, EMURX_ST_DOT1Q_TOO_SHORT);
    first(st, t2, EMURX_ST_TOO_MANY_DOT1Q);
#if EMURX_DWFIELDS
    r.vlan0 = g0 ? (W12 & 0xffff0fffu) : 0u;
    r.vlan1 = g1 ? (W16 & 0xffff0fffu) : 0u;
#else
    r.vlan0 = g0 ? (be32(s, 12) & 0xffff0fffu) : 0u;
    r.vlan1 = g1 ? (be32(s, 16) & 0xffff0fffu) : 0u;
#endif
    if (st != EMURX_ST_OK) { fail(r, st); return; }
    if (ppp0 || ppp1) { invoke(r, EMURX_CB_PPP, cb_mask); return; }
    const uint32_t offset = 14 + (g0 ? 4u : 0u) + (g1 ? 4u : 0u);
    const uint32_t et = g1 ? e2 : g0 ? e1 : e0;

    uint32_t l4 = 0, l4len = 0, nh = 0, pcs = 0;  // the L4 tail's inputs
    bool v6 = false;
    if (et == 0x0800) {  // IPv4
        r.l3 = offset;
#if EMURX_DWFIELDS
        // version / IHL, total length, flags / fragment offset and protocol from the header's
        // first three words (the dwords its checksum reads again) instead of six byte reads
        const uint32_t H0 = le32(s, offset), H4 = le32(s, offset + 4), H8 = le32(s, offset + 8);
        const uint32_t b0 = H0 & 0xff, totlen = (((H0 >> 16) & 0xff) << 8) | (H0 >> 24),
                       frag = (((H4 >> 16) & 0xff) << 8) | (H4 >> 24);
#else
        const uint32_t b0 = s.u8(offset), frag = be16(s, offset + 6), totlen = be16(s, offset + 2);
#endif
        const uint32_t hdr = (b0 & 0xf) << 2;
        first(st, len < offset + 20, EMURX_ST_IPV4_TOO_SHORT);
        first(st, (b0 >> 4) != 4, EMURX_ST_IPV4_HDR_TOO_SHORT);
        first(st, (frag & 0x3fff) != 0, EMURX_ST_IPV4_FRAGMENT);
        first(st, hdr < 20, EMURX_ST_IPV4_HDR_TOO_SHORT);
        first(st, len < offset + hdr, EMURX_ST_IPV4_HDR_TOO_SHORT);
        first(st, len < ((offset + totlen) & 0xffff), EMURX_ST_IPV4_TOO_SHORT);
        // the header sum: straight-line for the usual 20 bytes (a failed frame's value is unused)
        const uint32_t th = hdr == 20 ? s.template sum_fixed<20>(offset) : s.sum(offset, st == EMURX_ST_OK ? hdr : 0u);
        const bool hok = csum_ok(th, s.at(offset), 0);
        first(st, !hok, EMURX_ST_IPV4_CS);
        if (st != EMURX_ST_OK) { fail(r, st); return; }
        l4len = (totlen - hdr) & 0xffff;
        l4 = offset + hdr;
#if EMURX_DWFIELDS
        nh = (H8 >> 8) & 0xff;
#else
        nh = s.u8(offset + 9);
#endif
        pcs = be_domain(s.template sum_fixed<8>(offset + 12), s.at(offset + 12)) + nh + l4len;  // src, dst, 0|proto, len
    } else if (et == 0x86DD) {  // IPv6
        r.l3 = offset;
        const uint32_t plen = be16(s, offset + 4);
        first(st, len < offset + 40, EMURX_ST_IPV6_TOO_SHORT);
        first(st, (s.u8(offset) >> 4) != 6, EMURX_ST_IPV6_TOO_SHORT);
        first(st, len < ((offset + 40 + plen) & 0xffff), EMURX_ST_IPV6_TOO_SHORT);
        first(st, s.u8(offset + 7) == 0, EMURX_ST_IPV6_HOPLIMIT);
        if (st != EMURX_ST_OK) { fail(r, st); return; }
        uint32_t osize = 0;
        l4 = offset + 40;
        l4len = plen;
        nh = s.u8(offset + 6);
        for (;;) {  // extension headers (parser.go:886-931): rare, kept as Go's loop
            const bool ext = nh == 0 || nh == 60 || nh == 43 || nh == 51 || nh == 50 || nh == 135 ||
                             nh == 139 || nh == 140;
            if (!ext) break;
            if (l4len < 8) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if (l4 + 2 > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
            const uint32_t hl = (s.u8(l4 + 1) << 3) + 8;
            if (l4len < hl) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if (l4 + hl > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
            const uint32_t nnh = s.u8(l4);
            if (!ipv6_options(s, l4 + 2, (int)hl - 2, r.flags)) { fail(r, EMURX_ST_PANIC_IPV6_OPT); return; }
            nh = nnh;
            l4len -= hl;
            osize += hl;
            l4 += hl;
        }
        first(st, nh == 44, EMURX_ST_IPV6_FRAGMENT);
        first(st, nh == 194, EMURX_ST_IPV6_JUMBO);
        first(st, nh == 59, EMURX_ST_IPV6_EMPTY);
        if (st != EMURX_ST_OK) { fail(r, st); return; }
        v6 = true;
        pcs = be_domain(s.template sum_fixed<32>(offset + 8), s.at(offset + 8)) + ((plen - osize) & 0xffff) + nh;  // src, dst, len, 0|nh
    } else {
        // EAPOL, ARP (ARPHeaderSize 28), PPPoE, anything else
        const bool eap = et == 0x888E, arp = et == 0x0806;
        first(st, eap && len < offset + 4, EMURX_ST_EAPOL_TOO_SHORT);
        first(st, arp && len < offset + 28, EMURX_ST_ARP_TOO_SHORT);
        first(st, !eap && !arp && !is_ppp(et), EMURX_ST_L3_UNSUPPORTED);
        if (st != EMURX_ST_OK) { fail(r, st); return; }
        if (eap || arp) r.l3 = offset;
        invoke(r, eap ? EMURX_CB_EAPOL : arp ? EMURX_CB_ARP : EMURX_CB_PPP, cb_mask);
        return;
    }
    // IPv4 and IPv6 share parsePacketL4 (and its checksum span): one pass for a wave that
    // holds both
    r.l4 = l4;
    parse_l4_flat(s, len, r, nh, pcs, l4len, v6, cb_mask);
}

// ---------------------------------------------------------------------------------------
// Wave-cooperative L4 checksums for the WinSrc path (long spans, IMIX / jumbo frames).  The
// wave's deferred spans are dealt to its four 16-lane rows in lane order, balanced by their
// round counts, and each row walks its spans one after the other, 16 lanes x kCoopVec
// consecutive vectors of one span per round (coalesced 1 KiB row loads, no per-vector span
// search); a round's row total is folded by four DPP row shifts and added once into the span's
// LDS word; the owner lane settles its outcome.  Replaces a per-lane serial walk of up to ~90
// dependent loads.  Called with the wave converged.  4 vectors per lane per round measured
// best (2: +22 %, 8: +56 % on config E).
// ---------------------------------------------------------------------------------------
constexpr uint32_t kCoopVec = 4;
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return wave_reduce(v, [](uint32_t x, uint32_t y) { return x + y; });
}
__device__ __forceinline__ void settle_deferred(Rec& r, bool ok) {
    if (ok) return;
    const uint32_t st = r.dfail & 0xffffu;
    if (st == EMURX_ST_ICMPV4_CS || st == EMURX_ST_UDP_CS) r.l7 = 0;  // Go sets L7 after the check
    fail(r, st);
}
// vector k of a span of nv vectors (bytes [h, t) of the first / last)
__device__ __forceinline__ uint32_t span_sum(const uint4& x, uint32_t nv, int h, int t, uint32_t k) {
    if (k >= nv) return 0;
    return sad_vec_masked(x, k == 0 ? h : 0, k == nv - 1 ? t : 16, 0);
}
__device__ __forceinline__ uint32_t dpp_row_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    return v;  // lane 15 of each row: the row's total
}
#ifndef EMURX_COOP_NT
#define EMURX_COOP_NT 0
#endif
// The wave's spans [span, span + n) (lanes with mine set) summed by its four 16-lane rows in
// the dword form of glb_sum (sad of 16-bit halves, bytes outside the span masked): returns this
// lane's sum (0 when not mine).  wsum: kWave words of LDS owned by the wave.  Called converged.
__device__ __forceinline__ uint32_t coop_span_sum(const uint8_t* span, uint32_t n, bool mine, uint32_t* wsum) {
    constexpr uint32_t kRound = 16 * kCoopVec;  // vectors of one span per row round
    const uint32_t lane = lane_id(), l16 = lane & 15, row = lane >> 4;
    mine = mine && n != 0;
    const uint64_t mm = __ballot(mine);
    if (!mm) return 0;
    const uintptr_t a = (uintptr_t)span, e = a + n;
    const uint32_t nv = mine ? (uint32_t)((((e + 15) & ~(uintptr_t)15) - (a & ~(uintptr_t)15)) >> 4) : 0u;
    const uint32_t rounds = (nv + kRound - 1) / kRound;
    uint32_t incl = rounds;
#pragma unroll
    for (uint32_t o = 1; o < kWave; o <<= 1) {
        const uint32_t up = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += up;
    }
    const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    // row of this lane's span: its rounds' midpoint in the wave's total, in quarters
    const uint32_t g = mine ? min(3u, (uint32_t)(((uint64_t)(2 * incl - rounds) * 4) / (2 * (uint64_t)R))) : 4u;
    uint64_t rm = 0;  // the spans of this lane's row (lanes in order)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t b = __ballot(g == k);
        if (row == k) rm = b;
    }
    const uintptr_t a16 = a & ~(uintptr_t)15;
    const uint32_t blo = (uint32_t)a16, bhi = (uint32_t)(a16 >> 32);
    const uint32_t geo = nv | ((uint32_t)(a & 15) << 16) | ((16u - ((0u - (uint32_t)e) & 15)) << 24);
    wsum[lane] = 0;
    uint32_t j = rm ? (uint32_t)__ffsll((long long)rm) - 1 : 64u, c = 0;  // the row's current span, round
    for (;;) {  // wave-uniform: until every row has walked its spans
        if (!__ballot(j < 64)) break;
        const uint32_t src_lane = j < 64 ? j : 0u;
        const uint32_t gj = (uint32_t)__shfl((int)geo, (int)src_lane);
        const uint32_t lo = (uint32_t)__shfl((int)blo, (int)src_lane), hi = (uint32_t)__shfl((int)bhi, (int)src_lane);
        const uint8_t* src = reinterpret_cast<const uint8_t*>(((uintptr_t)hi << 32) | lo);
        const uint32_t nvj = j < 64 ? (gj & 0xffff) : 0u;
        uint4 x[kCoopVec];
#pragma unroll
        for (uint32_t k = 0; k < kCoopVec; ++k) {
            const uint32_t v = c * kRound + k * 16 + l16;
#if EMURX_COOP_NT  // build variant (A/B): the span bytes are read once, never again
            if (v < nvj) {
                const emurx_v4u y = __builtin_nontemporal_load((const __attribute__((address_space(1))) emurx_v4u*)(src + 16 * v));
                x[k] = make_uint4(y.x, y.y, y.z, y.w);
            } else {
                x[k] = make_uint4(0, 0, 0, 0);
            }
#else
            x[k] = v < nvj ? gld16(src + 16 * v) : make_uint4(0, 0, 0, 0);
#endif
        }
        uint32_t part = 0;
#pragma unroll
        for (uint32_t k = 0; k < kCoopVec; ++k)
            part += span_sum(x[k], nvj, (int)((gj >> 16) & 0xff), (int)(gj >> 24), c * kRound + k * 16 + l16);
        const uint32_t tot = dpp_row_sum(part);
        if (l16 == 15 && j < 64 && tot) atomicAdd(&wsum[j], tot);
        if (j < 64 && ++c * kRound >= nvj) {  // the span is done: the row's next one
            c = 0;
            const uint64_t rest = j < 63 ? rm & (~0ull << (j + 1)) : 0ull;
            j = rest ? (uint32_t)__ffsll((long long)rest) - 1 : 64u;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return mine ? wsum[lane] : 0u;
}
// the rx window path's deferred L4 checksums (r.dstart / r.dlen of each lane's frame f)
__device__ __forceinline__ void coop_checksum_rows(Rec& r, const uint8_t* f, uint32_t* wsum) {
    const bool mine = r.dlen != 0;
    if (!__ballot(mine)) return;
    const uint32_t T = coop_span_sum(f + r.dstart, r.dlen, mine, wsum);
    if (mine) {
        settle_deferred(r, csum_ok(T, r.dfail >> 16, r.dpcs));  // parity of the span's start
        r.dlen = 0;
    }
}

// ---------------------------------------------------------------------------------------
// Namespace / Client lookups (GetNs thread_ctx.go:777-784, CLookupBy* ns_ctx.go:262-329)
// over the bucketed tables of emurx_tables.h.  A frame's Namespace bucket and its client
// bucket both follow from the parsed tunnel key, so classify() issues the two 64-byte
// bucket reads together and resolves them afterwards; overflow buckets are rare.
// ---------------------------------------------------------------------------------------
struct Bucket {
    uint4 s[4];
};
__device__ __forceinline__ Bucket ld_bucket(const uint32_t* tab, uint32_t b) {
    const uint32_t* p = tab + (size_t)b * EMURX_BUCKET_WORDS;
    return Bucket{{gld16(p), gld16(p + 4), gld16(p + 8), gld16(p + 12)}};
}

// Lookups stop at the first bucket holding an empty slot.  A key sits at most once in a
// table and the host rebuilds the tables without holes (bucket_put, emurx_api.cpp), so "a
// matching slot anywhere in the bucket" equals the in-order scan and slot order is free.
// ns slot {vport | ns_plugins << 16, vlan0, vlan1, ns_id} -> (ns_id, ns plugin mask)
__device__ __forceinline__ uint2 resolve_ns(const emurx_dev_tables& T, uint32_t b, Bucket e, uint32_t w0, uint32_t w1,
                            uint32_t w2) {
    {  // the home bucket's first slot alone: the common hit, a uniform early exit
        const uint4 x = e.s[0];
        if (x.w != EMURX_EMPTY && (x.x & 0xffffu) == w0 && x.y == w1 && x.z == w2) return make_uint2(x.w, x.x >> 16);
    }
    for (uint32_t n = 0;;) {
        bool hole = false;
        uint2 hit = make_uint2(EMURX_ID_NONE, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 x = e.s[k];
            hole |= x.w == EMURX_EMPTY;
            if (x.w != EMURX_EMPTY && (x.x & 0xffffu) == w0 && x.y == w1 && x.z == w2) hit = make_uint2(x.w, x.x >> 16);
        }
        if (hit.x != EMURX_ID_NONE || hole || ++n > T.ns_mask) return hit;
        b = (b + 1) & T.ns_mask;
        e = ld_bucket(T.ns_tab, b);
    }
}
// mac slot {ns_id, mac[0..3], mac[4..5] | client_plugins << 16, client_id} -> (cid, plugins)
__device__ __forceinline__ uint2 resolve_mac(const emurx_dev_tables& T, uint32_t b, Bucket e, uint32_t ns, uint32_t lo,
                             uint32_t hi) {
    {
        const uint4 x = e.s[0];
        if (x.w != EMURX_EMPTY && x.x == ns && x.y == lo && (x.z & 0xffffu) == hi) return make_uint2(x.w, x.z >> 16);
    }
    for (uint32_t n = 0;;) {
        bool hole = false;
        uint2 hit = make_uint2(EMURX_ID_NONE, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 x = e.s[k];
            hole |= x.w == EMURX_EMPTY;
            if (x.w != EMURX_EMPTY && x.x == ns && x.y == lo && (x.z & 0xffffu) == hi) hit = make_uint2(x.w, x.z >> 16);
        }
        if (hit.x != EMURX_ID_NONE || hole || ++n > T.mac_mask) return hit;
        b = (b + 1) & T.mac_mask;
        e = ld_bucket(T.mac_tab, b);
    }
}
// IP slots carry the client's MAC and plugin mask: {cid, mac_lo, mac_hi | plugins << 16}
struct IpHit {
    uint32_t cid, mlo, mhip;
};
// ip4 slot {ns_id, ip, mac_lo, mac_hi | plugins << 16} {0, 0, 0, client_id}, 2 per bucket
__device__ __forceinline__ IpHit resolve_ip4(const emurx_dev_tables& T, uint32_t b, Bucket e, uint32_t ns, uint32_t ip) {
    {
        const uint4 x = e.s[0], y = e.s[1];
        if (y.w != EMURX_EMPTY && x.x == ns && x.y == ip) return IpHit{y.w, x.z, x.w};
    }
    for (uint32_t n = 0;;) {
        bool hole = false;
        IpHit hit{EMURX_ID_NONE, 0, 0};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 x = e.s[2 * k], y = e.s[2 * k + 1];
            hole |= y.w == EMURX_EMPTY;
            if (y.w != EMURX_EMPTY && x.x == ns && x.y == ip) hit = IpHit{y.w, x.z, x.w};
        }
        if (hit.cid != EMURX_ID_NONE || hole || ++n > T.ip4_mask) return hit;
        b = (b + 1) & T.ip4_mask;
        e = ld_bucket(T.ip4_tab, b);
    }
}
// ip6 slot {ns_id, ip[0..3], ip[4..7], ip[8..11]} {ip[12..15], mac_lo, mac_hi | plugins << 16,
// client_id}, 2 per bucket
__device__ __forceinline__ IpHit resolve_ip6(const emurx_dev_tables& T, uint32_t b, Bucket e, uint32_t ns, const uint32_t w[4]) {
    for (uint32_t n = 0;;) {
        bool hole = false;
        IpHit hit{EMURX_ID_NONE, 0, 0};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 x = e.s[2 * k], y = e.s[2 * k + 1];
            hole |= y.w == EMURX_EMPTY;
            if (y.w != EMURX_EMPTY && x.x == ns && x.y == w[0] && x.z == w[1] && x.w == w[2] && y.x == w[3])
                hit = IpHit{y.w, y.y, y.z};
        }
        if (hit.cid != EMURX_ID_NONE || hole || ++n > T.ip6_mask) return hit;
        b = (b + 1) & T.ip6_mask;
        e = ld_bucket(T.ip6_tab, b);
    }
}

__device__ __forceinline__ void set_lk(Rec& r, uint32_t lk) {
    r.flags = (r.flags & ~EMURX_FLAG_LK_MASK) | (lk << EMURX_FLAG_LK_SHIFT);
}
// client found -> client.PluginCtx.Get(<plugin>) where the handler checks it
__device__ __forceinline__ void client_result(Rec& r, uint32_t cid, uint32_t cplugins, uint32_t plug,
                                              bool check) {
    if (cid == EMURX_ID_NONE) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
    r.cl = cid;
    if (check && !(cplugins & (1u << plug))) { set_lk(r, EMURX_LK_CLIENT_NO_PLUGIN); return; }
    set_lk(r, EMURX_LK_CLIENT);
}
// client info slot {cid, plugins, ra, ra_prefix[0..3], ra_prefix[4..7], has_ctx, 0, 0} of a
// client id (emurx_tables.h ci table, 2 per bucket); zeros when absent
struct CInfo {
    uint32_t plugins, ra, ra0, ra1, ctx;
};
__device__ __forceinline__ CInfo client_info(const emurx_dev_tables& T, uint32_t cid) {
    CInfo c{0, 0, 0, 0, 0};
    if (cid == EMURX_ID_NONE) return c;
    for (uint32_t b = emurx_ci_hash(cid) & T.ci_mask, n = 0; n <= T.ci_mask; b = (b + 1) & T.ci_mask, ++n) {
        const Bucket e = ld_bucket(T.ci_tab, b);
        bool hole = false;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 x = e.s[2 * k], y = e.s[2 * k + 1];
            hole |= y.w == EMURX_EMPTY;
            if (y.w != EMURX_EMPTY && x.x == cid) return CInfo{x.y, x.z, x.w, y.x, y.y};
        }
        if (hole) break;
    }
    return c;
}
// CClient.IsUnicastToMe client_ctx.go:389-398 (frames here are always > 6 bytes) compares the
// frame's destination with the client's MAC, which the IP slots carry (IpHit)

// Go 1.18 net.IP.IsLinkLocalUnicast / IsGlobalUnicast for a 16-byte address (words LE)
__device__ __forceinline__ bool ip6_local_or_global(const uint32_t w[4]) {
    uint32_t b0 = w[0] & 0xff, b1 = (w[0] >> 8) & 0xff;
    bool v4in6 = w[0] == 0 && w[1] == 0 && (w[2] & 0xffff) == 0 && (w[2] >> 16) == 0xffffu;
    if (v4in6) {
        uint32_t v = w[3], c0 = v & 0xff, c1 = (v >> 8) & 0xff;
        bool ll = c0 == 169 && c1 == 254;
        if (ll) return true;
        if (v == 0xffffffffu || v == 0 || c0 == 127 || (c0 & 0xf0) == 0xe0) return false;
        return true;
    }
    bool ll = b0 == 0xfe && (b1 & 0xc0) == 0x80;
    if (ll) return true;
    if ((w[0] | w[1] | w[2] | w[3]) == 0) return false;                      // unspecified
    if (w[0] == 0 && w[1] == 0 && w[2] == 0 && w[3] == 0x01000000u) return false;  // ::1
    if (b0 == 0xff) return false;                                            // multicast
    return true;
}
// PluginDhcpNs.GetMacFromDhcp dhcp.go:863-891 + DHCPv4.DecodeFromBytes dhcpv4.go:125-172
template <class S>
__device__ bool dhcp_chaddr(const S& s, uint32_t len, const Rec& r, uint32_t& lo, uint32_t& hi) {
    uint32_t d = r.l7, dlen = r.l7len;
    if (dlen < 240) return false;
    if (((d + dlen) & 0xffff) < d || d + dlen > len) return false;
    if (be32(s, d + 236) != 0x63825363u) return false;
    if (dlen > 240) {
        uint32_t o = d + 240;
        int stop = (int)dlen - 240, start = 0;
        while (start < stop) {
            uint32_t t = s.u8(o + start);
            if (t == 255) break;
            if (t == 0) { start++; continue; }
            if (stop - start < 2) return false;
            int l = (int)s.u8(o + start + 1);
            if (l > stop - start - 2) return false;
            start += l + 2;
        }
    }
    if (s.u8(d + 1) != 1 || s.u8(d + 2) != 6) return false;
    lo = le32(s, d + 28);
    hi = s.u8(d + 32) | (s.u8(d + 33) << 8);
    return true;
}

// The frame's c5tuplekey (fillv4tuple / fillv6tuple src/emu/plugins/transport/
// client_ctx.go:720-765) and the TCP flags byte the new-flow check reads.
struct Tuple {
    uint32_t v6, proto, ports, flags;  // ports: sport, dport as on the wire (4 bytes LE)
    uint32_t a[4], d[4];               // src / dst words LE (IPv4: a[0], d[0])
};
template <class S>
__device__ __forceinline__ Tuple get_tuple(const S& s, uint32_t len, const Rec& r) {
    Tuple t{};
    const uint32_t L3 = r.l3, L4 = r.l4;
    t.ports = le32(s, L4);  // UDPHeader(p[L4:L4+4])
    if ((s.u8(L3) >> 4) == 4) {  // IPv4Header(p[L3:L3+20]).Version()
        t.proto = s.u8(L3 + 9);
        t.a[0] = le32(s, L3 + 12);
        t.d[0] = le32(s, L3 + 16);
    } else {
        t.v6 = 1;
        t.proto = r.nh;  // ps.NextHeader
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            t.a[k] = le32(s, L3 + 8 + 4 * k);
            t.d[k] = le32(s, L3 + 24 + 4 * k);
        }
    }
    // a flags byte past the frame is read as 0 here (stale mbuf bytes in Go)
    t.flags = (L4 + 13 < len) ? s.u8(L4 + 13) : 0u;
    return t;
}
// TransportCtx.handleRxPacket client_ctx.go:912-969: the tuple in the client's flow map,
// else the new-flow checks of handleRxTcpNewFlow / handleRxUdpNewFlow (:829-904) up to OnAccept
__device__ __forceinline__ uint32_t flow_probe(const emurx_dev_tables& T, const Tuple& t, uint32_t cid) {
    const uint32_t proto = t.proto, ports = t.ports;
    if (!t.v6) {
        const uint32_t src = t.a[0], dst = t.d[0];
        for (uint32_t b = emurx_ft4_hash(cid, src, dst, ports, proto) & T.ft4_mask, k = 0; k <= T.ft4_mask;
             ++k, b = (b + 1) & T.ft4_mask) {
            const Bucket e = ld_bucket(T.ft4_tab, b);
            const uint4 x0 = e.s[0], x1 = e.s[1], y0 = e.s[2], y1 = e.s[3];
            if (x0.x == cid && x0.y == src && x0.z == dst && x0.w == ports && x1.x == proto && x1.w != EMURX_EMPTY)
                return x1.w;
            if (y0.x == cid && y0.y == src && y0.z == dst && y0.w == ports && y1.x == proto && y1.w != EMURX_EMPTY)
                return y1.w;
            if (x1.w == EMURX_EMPTY || y1.w == EMURX_EMPTY) break;
        }
    } else {
        for (uint32_t b = emurx_ft6_hash(cid, t.a[0], t.a[1], t.a[2], t.a[3], t.d[0], t.d[1], t.d[2], t.d[3], ports,
                                         proto) & T.ft6_mask, k = 0;
             k <= T.ft6_mask; ++k, b = (b + 1) & T.ft6_mask) {
            const Bucket e = ld_bucket(T.ft6_tab, b);
            if (e.s[3].w == EMURX_EMPTY) break;
            if (e.s[0].x == cid && e.s[0].y == t.a[0] && e.s[0].z == t.a[1] && e.s[0].w == t.a[2] &&
                e.s[1].x == t.a[3] && e.s[1].y == t.d[0] && e.s[1].z == t.d[1] && e.s[1].w == t.d[2] &&
                e.s[2].x == t.d[3] && e.s[2].y == ports && e.s[2].z == proto)
                return e.s[3].w;
        }
    }
    // a new flow: handleRxTcpNewFlow needs a bare SYN (GetFlags() & 0x3F == 0x2)
    if (proto == 6 && (t.flags & 0x3f) != 0x2) return EMURX_FLOW_NO_SYN;
    const uint32_t dport = ((ports >> 16) & 0xff) << 8 | (ports >> 24);
    const uint32_t key = dport | ((proto == 6 ? 6u : 17u) << 16);  // lookupServerPort(dst, TCP|UDP)
    for (uint32_t b = emurx_srv_hash(cid, key) & T.srv_mask, k = 0; k <= T.srv_mask; ++k, b = (b + 1) & T.srv_mask) {
        const Bucket e = ld_bucket(T.srv_tab, b);
        bool hole = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            hole |= e.s[j].w == EMURX_EMPTY;
            if (e.s[j].w != EMURX_EMPTY && e.s[j].x == cid && e.s[j].y == key) return EMURX_FLOW_NEW;
        }
        if (hole) break;
    }
    return EMURX_FLOW_NO_SERVER;
}

// the plugin whose PluginCtx each callback checks, a nibble per callback in one immediate (a
// __constant__ byte table indexed per lane costs a vector load behind the bucket reads)
constexpr uint8_t kCbPluginTab[EMURX_NUM_CB] = {
    EMURX_PLUG_ARP, EMURX_PLUG_ICMP, EMURX_PLUG_IGMP, EMURX_PLUG_DHCP, EMURX_PLUG_DHCPSRV,
    EMURX_PLUG_DHCPV6, EMURX_PLUG_MDNS, EMURX_PLUG_TRANSPORT, EMURX_PLUG_TRANSPORT,
    EMURX_PLUG_IPV6, EMURX_PLUG_DOT1X, EMURX_PLUG_PPP};
constexpr uint64_t cb_plugin_packed() {
    uint64_t v = 0;
    for (int i = 0; i < EMURX_NUM_CB; ++i) v |= (uint64_t)kCbPluginTab[i] << (4 * i);
    return v;
}
static_assert(EMURX_NUM_CB <= 16 && EMURX_NUM_PLUG <= 16, "a nibble per callback");
__device__ __forceinline__ uint32_t cb_plugin(uint32_t cb) {
    return (uint32_t)(cb_plugin_packed() >> (4 * (cb & 15))) & 15u;
}

// what a callback's client rule looks up, decided from the frame alone (before the
// Namespace is known, so both probes can be issued together)
enum Key : uint32_t {
    kNsLevel = 0,  // no client lookup (igmp, mdns, arp reply, icmpv6 non-echo)
    kNoClient,     // the rule fails before any lookup (dhcp broadcast without chaddr, ...)
    kFirst,        // ns.GetFirstClient (dhcpsrv broadcast, eapol PAE group address)
    kMac,          // CLookupByMac(kw[0..1])
    kEui,          // CLookupByIPv6LocalGlobal, EUI-64 form: MAC from the address + prefix rule
    kIp4,          // CLookupByIPv4(kw[0])
    kIp6,          // CLookupByIPv6(kw[0..3])
};

// The lookup key of a frame's callback rule, decided from the frame alone (before the
// Namespace is known, so both probes can be issued together; and, in the partitioned path,
// on the GPU that received the frame, with the probes on the Namespace's owner).
struct LKey {
    uint32_t key;    // enum Key
    uint32_t kw[4];  // kMac: MAC lo, hi; kIp4: address; kIp6 / kEui: the IPv6 destination
    uint32_t dlo, dhi;  // destination MAC (IsUnicastToMe)
    uint32_t mc6;    // icmpv6: the IPv6 source starts with 0xff
};
template <class S>
__device__ __forceinline__ LKey make_key(const S& s, uint32_t len, const Rec& r) {
    const uint32_t cb = r.proto;
    LKey k;
    k.dlo = le32(s, 0);
#if EMURX_DWFIELDS
    if constexpr (std::is_same<S, LdsSrc>::value) k.dhi = le32(s, 4) & 0xffffu;  // p[4:6] from a dword word
    else k.dhi = s.u8(4) | (s.u8(5) << 8);
#else
    k.dhi = s.u8(4) | (s.u8(5) << 8);  // p[0:6]
#endif
    k.mc6 = 0;
    const bool bcast = k.dlo == 0xffffffffu && k.dhi == 0xffffu;
    k.key = kMac;
    k.kw[0] = k.dlo; k.kw[1] = k.dhi; k.kw[2] = 0; k.kw[3] = 0;
    switch (cb) {
    case EMURX_CB_ARP:  // arp.go:904-949: request -> IPv4 of the ARP target
        if (be16(s, r.l3 + 6) == 1) { k.key = kIp4; k.kw[0] = le32(s, r.l3 + 24); }
        else k.key = kNsLevel;
        break;
    case EMURX_CB_ICMP:  // icmp.go:396-427: IPv4 destination, then IsUnicastToMe
        k.key = kIp4; k.kw[0] = le32(s, r.l3 + 16);
        break;
    case EMURX_CB_IGMP:
    case EMURX_CB_MDNS:
        k.key = kNsLevel;
        break;
    case EMURX_CB_DHCP:  // dhcp.go:893-917: broadcast -> chaddr
        if (bcast && !dhcp_chaddr(s, len, r, k.kw[0], k.kw[1])) k.key = kNoClient;
        break;
    case EMURX_CB_DHCPSRV:  // dhcpsrv.go:1798-1826: broadcast -> GetFirstClient
        if (bcast) k.key = kFirst;
        break;
    case EMURX_CB_EAPOL:  // dot1x.go:624-650: 01:80:c2:00:00:03 -> GetFirstClient
        if (k.dlo == 0x00c28001u && k.dhi == 0x0300u) k.key = kFirst;
        break;
    case EMURX_CB_ICMPV6: {  // ipv6.go:465-540: echo request -> CLookupByIPv6LocalGlobal(dst)
        if (be16(s, r.l4) != 0x8000u) { k.key = kNsLevel; break; }
        if (r.l3 + 40 > len) { k.key = kNoClient; break; }
        for (int j = 0; j < 4; ++j) k.kw[j] = le32(s, r.l3 + 24 + 4 * j);
        if (!ip6_local_or_global(k.kw)) { k.key = kNoClient; break; }
        // ExtractOnlyMac client_ctx.go:314-329
        k.key = (((k.kw[2] >> 24) & 0xff) == 0xff && (k.kw[3] & 0xff) == 0xfe) ? kEui : kIp6;
        k.mc6 = s.u8(r.l3 + 8) == 0xff;
        break;
    }
    default:  // dhcpv6, ppp, tcp, udp: MAC[dst] (plugin_transport.go:83-115, ...)
        break;
    }
    // zero keys never match (MACKey / Ipv4Key / Ipv6Key IsZero, ns_ctx.go:262-329)
    if (k.key == kMac && k.kw[0] == 0 && k.kw[1] == 0) k.key = kNoClient;
    if (k.key == kIp4 && k.kw[0] == 0) k.key = kNoClient;
    if (k.key == kIp6 && (k.kw[0] | k.kw[1] | k.kw[2] | k.kw[3]) == 0) k.key = kNoClient;
    if (k.key == kEui) {  // the MAC of an EUI-64 address; a zero MAC never matches
        const uint32_t lo = ((k.kw[2] & 0xff) ^ 2) | (((k.kw[2] >> 8) & 0xff) << 8) | (((k.kw[2] >> 16) & 0xff) << 16) |
                            (((k.kw[3] >> 8) & 0xff) << 24);
        const uint32_t hi = ((k.kw[3] >> 16) & 0xff) | ((k.kw[3] >> 24) << 8);
        if (lo == 0 && hi == 0) k.key = kNoClient;
    }
    return k;
}

// The two bucket reads of a frame's lookups, issued together: its Namespace bucket (loaded
// here) and the first bucket of its client table (ctab == nullptr: the rule reads none).
struct Probe {
    uint32_t nb, cbk, mlo, mhi;  // mlo / mhi: the MAC probed for kMac / kEui
    const uint32_t* ctab;
    Bucket ne;
};
#ifndef EMURX_UNIHASH
#define EMURX_UNIHASH 0
#endif
__device__ __forceinline__ Probe probe_issue(const emurx_dev_tables& T, const Rec& r, const LKey& k) {
    Probe p;
    const uint32_t key = k.key;
    p.mlo = k.kw[0];
    p.mhi = k.kw[1];
    if (key == kEui) {
        p.mlo = ((k.kw[2] & 0xff) ^ 2) | (((k.kw[2] >> 8) & 0xff) << 8) | (((k.kw[2] >> 16) & 0xff) << 16) |
                (((k.kw[3] >> 8) & 0xff) << 24);
        p.mhi = ((k.kw[3] >> 16) & 0xff) | ((k.kw[3] >> 24) << 8);
    }
#if EMURX_UNIHASH
    // a wave whose frames share one CTunnelKey (one port's untagged or one-VLAN traffic) or
    // one MAC key hashes it once, on the scalar unit (build variant for A/B)
    const uint32_t u0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.vport),
                   u1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.vlan0),
                   u2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.vlan1);
    const bool tku = __ballot(r.vport != u0 || r.vlan0 != u1 || r.vlan1 != u2) == 0;
    uint32_t tk;
    if (tku) tk = emurx_tk_hash(u0, u1, u2);  // wave-uniform branch: scalar arithmetic
    else tk = emurx_tk_hash(r.vport, r.vlan0, r.vlan1);
#else
    const uint32_t tk = emurx_tk_hash(r.vport, r.vlan0, r.vlan1);  // CTunnelKey words
#endif
    p.nb = tk & T.ns_mask;
    p.ne = ld_bucket(T.ns_tab, p.nb);
    p.cbk = 0;
    p.ctab = nullptr;
    // The three table bases as SGPR values selected per lane: left to itself the compiler
    // turns "this lane's table pointer" into a vector load from the kernarg segment at a
    // per-lane offset, one more dependent memory trip before the client bucket's address
    uintptr_t tm = (uintptr_t)T.mac_tab, t4 = (uintptr_t)T.ip4_tab, t6 = (uintptr_t)T.ip6_tab;
    asm volatile("" : "+s"(tm), "+s"(t4), "+s"(t6));
    if (key == kMac || key == kEui) {
#if EMURX_UNIHASH
        const uint32_t m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.mlo),
                       m1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.mhi);
        const bool mu = tku && __ballot(p.mlo != m0 || p.mhi != m1) == 0;
        if (mu) p.cbk = emurx_mac_hash((uint32_t)__builtin_amdgcn_readfirstlane((int)tk), m0, m1) & T.mac_mask;
        else p.cbk = emurx_mac_hash(tk, p.mlo, p.mhi) & T.mac_mask;
#else
        p.cbk = emurx_mac_hash(tk, p.mlo, p.mhi) & T.mac_mask;
#endif
        p.ctab = reinterpret_cast<const uint32_t*>(tm);
    } else if (key == kIp4) {
        p.cbk = emurx_ip4_hash(tk, k.kw[0]) & T.ip4_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(t4);
    } else if (key == kIp6) {
        p.cbk = emurx_ip6_hash(tk, k.kw[0], k.kw[1], k.kw[2], k.kw[3]) & T.ip6_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(t6);
    }
    return p;
}

// GetNs + the callback's client rule, given the two buckets.  `flow(cid)` gives the transport
// flow decision of a tcp/udp frame whose client was found with the transport plugin.
template <class Flow>
__device__ __forceinline__ void resolve_done(const emurx_dev_tables& T, Rec& r, const LKey& k, const Probe& p,
                                             const Bucket& ce, Flow flow) {
    const uint32_t cb = r.proto, plug = cb_plugin(cb);
    const uint32_t key = k.key, cbk = p.cbk, mlo = p.mlo, mhi = p.mhi;
    // ---- GetNs + ns.PluginCtx.Get(plugin) ----
    const uint2 nsr = resolve_ns(T, p.nb, p.ne, r.vport, r.vlan0, r.vlan1);
    const uint32_t ns = nsr.x;
    if (ns == EMURX_ID_NONE) { set_lk(r, EMURX_LK_NO_NS); return; }
    r.ns = ns;
    if (!(nsr.y & (1u << plug))) { set_lk(r, EMURX_LK_NS_NO_PLUGIN); return; }

    // ---- the client rule ----
    switch (key) {
    case kNsLevel:
        set_lk(r, EMURX_LK_NS_LEVEL);
        return;
    case kNoClient:
        set_lk(r, EMURX_LK_NO_CLIENT);
        return;
    case kFirst: {
        const uint32_t cid = gld4(T.ns_info + 4 * ns + 1);
        client_result(r, cid, client_info(T, cid).plugins, plug, true);
        return;
    }
    case kIp4: {
        const IpHit h = resolve_ip4(T, cbk, ce, ns, k.kw[0]);
        if (cb == EMURX_CB_ARP) {
            client_result(r, h.cid, h.mhip >> 16, plug, true);
        } else {  // icmp: IsUnicastToMe against the MAC in the slot
            const bool me = h.mlo == k.dlo && (h.mhip & 0xffffu) == k.dhi;
            client_result(r, me ? h.cid : EMURX_ID_NONE, 0, plug, false);
        }
        return;
    }
    case kEui:
    case kIp6: {  // icmpv6 echo request
        uint32_t cid, clo, chi;  // the client and its MAC (IsUnicastToMe)
        if (key == kEui) {
            cid = resolve_mac(T, cbk, ce, ns, mlo, mhi).x;
            clo = mlo;  // the MAC table's key is the client's MAC
            chi = mhi;
            // CClient.IsValidPrefix client_ctx.go:279-295
            if (cid != EMURX_ID_NONE && !(k.kw[0] == 0x000080feu && k.kw[1] == 0)) {
                const CInfo c = client_info(T, cid);
                if (!((c.ra & 1u) && ((c.ra >> 8) & 0xff) == 64 && c.ra0 == k.kw[0] && c.ra1 == k.kw[1]))
                    cid = EMURX_ID_NONE;
            }
        } else {
            const IpHit h = resolve_ip6(T, cbk, ce, ns, k.kw);
            cid = h.cid;
            clo = h.mlo;
            chi = h.mhip & 0xffffu;
        }
        if (cid != EMURX_ID_NONE && !(clo == k.dlo && chi == k.dhi)) cid = EMURX_ID_NONE;
        if (cid != EMURX_ID_NONE && k.mc6) cid = EMURX_ID_NONE;
        client_result(r, cid, 0, plug, false);
        return;
    }
    default: {  // kMac
        const uint2 c = resolve_mac(T, cbk, ce, ns, mlo, mhi);
        client_result(r, c.x, c.y, plug, true);
        // transport: the client's TransportCtx decides (plugin_transport.go:109-114, :73-80)
        if ((cb == EMURX_CB_TCP || cb == EMURX_CB_UDP) &&
            ((r.flags & EMURX_FLAG_LK_MASK) >> EMURX_FLAG_LK_SHIFT) == EMURX_LK_CLIENT) {
            // GetTransportCtx() == nil -> the handler returns -1 (PluginTransClient :73-80);
            // the MAC slot carries the client's TransportCtx bit, so no client info is read
            r.flow = T.ft_on && (c.y & EMURX_CPL_CTX) ? flow(c.x) : EMURX_FLOW_NO_CTX;  // the MAC slot's ctx bit
        }
        return;
    }
    }
}

// The same outcome as resolve_done with far fewer divergent branches (EMURX_FLATRES, build
// variant for A/B): every table kind's answer from the first buckets by straight-line selects
// (the client bucket read as MAC, IPv4 and IPv6 slots at once: the lane's key kind picks one),
// probe chains past the first bucket behind one wave-uniform test (the sparse tables make them
// rare), the rule's outcome by selects, and the rules that read memory again (GetFirstClient,
// the EUI-64 RA-prefix check, the transport flow) behind wave-uniform "any lane" tests.  The
// divergent switch over key kinds in resolve_done costs its wave exec-mask bookkeeping for
// every kind present, which mixed traffic (config C) pays on every wave.
#ifndef EMURX_FLATRES
#define EMURX_FLATRES 0
#endif
__device__ __forceinline__ bool any_lane(bool c) { return __ballot(c) != 0; }
template <class Flow>
__device__ __forceinline__ void resolve_done_flat(const emurx_dev_tables& T, Rec& r, const LKey& k, const Probe& p,
                                                  const Bucket& ce, Flow flow) {
    const uint32_t cb = r.proto, plug = cb_plugin(cb), key = k.key;
    const uint32_t w0 = r.vport, w1 = r.vlan0, w2 = r.vlan1;
    // ---- first buckets, every view at once ----
    uint2 nsr = make_uint2(EMURX_ID_NONE, 0), mc = make_uint2(EMURX_ID_NONE, 0);
    IpHit i4{EMURX_ID_NONE, 0, 0}, i6{EMURX_ID_NONE, 0, 0};
    bool nhole = false, mhole = false, h4 = false, h6 = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 x = p.ne.s[j];
        nhole |= x.w == EMURX_EMPTY;
        if (x.w != EMURX_EMPTY && (x.x & 0xffffu) == w0 && x.y == w1 && x.z == w2) nsr = make_uint2(x.w, x.x >> 16);
    }
    const bool isMac = key == kMac || key == kEui, isIp4 = key == kIp4, isIp6 = key == kIp6;
    // the client views compare the Namespace id found above; a view no lane of the wave needs
    // is skipped (wave-uniform tests: a wave of one key kind computes one view)
    if (any_lane(isMac)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 y = ce.s[j];
            mhole |= y.w == EMURX_EMPTY;
            if (y.w != EMURX_EMPTY && y.x == nsr.x && y.y == p.mlo && (y.z & 0xffffu) == p.mhi) mc = make_uint2(y.w, y.z >> 16);
        }
    }
    if (any_lane(isIp4 || isIp6)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint4 x = ce.s[2 * j], y = ce.s[2 * j + 1];
            h4 |= y.w == EMURX_EMPTY;
            h6 |= y.w == EMURX_EMPTY;
            if (y.w != EMURX_EMPTY && x.x == nsr.x && x.y == k.kw[0]) i4 = IpHit{y.w, x.z, x.w};
            if (y.w != EMURX_EMPTY && x.x == nsr.x && x.y == k.kw[0] && x.z == k.kw[1] && x.w == k.kw[2] && y.x == k.kw[3])
                i6 = IpHit{y.w, y.y, y.z};
        }
    }
    // ---- chains past the first buckets (wave-uniform test; the loop resolvers walk on) ----
    const bool ns_more = nsr.x == EMURX_ID_NONE && !nhole;
    if (any_lane(ns_more) && ns_more) {
        const uint32_t b = (p.nb + 1) & T.ns_mask;
        nsr = resolve_ns(T, b, ld_bucket(T.ns_tab, b), w0, w1, w2);
    }
    const uint32_t ns = nsr.x;
    // the client probe needs the Namespace id: a lane whose Namespace came from its chain, or
    // whose client key lies past the first bucket, resolves its client from the start again
    const bool c_more = ns != EMURX_ID_NONE && (nsr.y & (1u << plug)) &&
                        (ns_more || (isMac && mc.x == EMURX_ID_NONE && !mhole) ||
                         (isIp4 && i4.cid == EMURX_ID_NONE && !h4) || (isIp6 && i6.cid == EMURX_ID_NONE && !h6));
    if (any_lane(c_more) && c_more) {
        if (isMac) mc = resolve_mac(T, p.cbk, ce, ns, p.mlo, p.mhi);
        else if (isIp4) i4 = resolve_ip4(T, p.cbk, ce, ns, k.kw[0]);
        else if (isIp6) i6 = resolve_ip6(T, p.cbk, ce, ns, k.kw);
    }
    // ---- the rule's client, by selects ----
    uint32_t cid = EMURX_ID_NONE, cpl = 0, clo = 0, chi = 0;
    bool check = true;
    if (isMac) { cid = mc.x; cpl = mc.y; clo = p.mlo; chi = p.mhi; }
    if (isIp4) { cid = i4.cid; cpl = i4.mhip >> 16; clo = i4.mlo; chi = i4.mhip & 0xffffu; }
    if (isIp6) { cid = i6.cid; clo = i6.mlo; chi = i6.mhip & 0xffffu; }
    const bool icmp4 = isIp4 && cb != EMURX_CB_ARP;
    if (icmp4 && !(clo == k.dlo && chi == k.dhi)) cid = EMURX_ID_NONE;  // IsUnicastToMe
    check = !(icmp4 || key == kEui || isIp6);
    const bool ns_ok = ns != EMURX_ID_NONE && (nsr.y & (1u << plug));
    // GetFirstClient (dhcpsrv / eapol) and the EUI-64 RA-prefix check read client info
    const bool first = ns_ok && key == kFirst;
    const bool eui = ns_ok && key == kEui && cid != EMURX_ID_NONE && !(k.kw[0] == 0x000080feu && k.kw[1] == 0);
    if (any_lane(first || eui)) {
        if (first) cid = gld4(T.ns_info + 4 * ns + 1);
        if (first || eui) {
            const CInfo c = client_info(T, cid);
            cpl = c.plugins;
            if (eui && !((c.ra & 1u) && ((c.ra >> 8) & 0xff) == 64 && c.ra0 == k.kw[0] && c.ra1 == k.kw[1]))
                cid = EMURX_ID_NONE;
        }
    }
    if ((key == kEui || isIp6) && cid != EMURX_ID_NONE && (!(clo == k.dlo && chi == k.dhi) || k.mc6)) cid = EMURX_ID_NONE;
    // ---- the outcome ----
    uint32_t lk = cid == EMURX_ID_NONE ? EMURX_LK_NO_CLIENT
                  : (check && !(cpl & (1u << plug))) ? EMURX_LK_CLIENT_NO_PLUGIN : EMURX_LK_CLIENT;
    if (key == kNsLevel) lk = EMURX_LK_NS_LEVEL;
    if (key == kNoClient) lk = EMURX_LK_NO_CLIENT;
    if (!(nsr.y & (1u << plug))) lk = EMURX_LK_NS_NO_PLUGIN;
    if (ns == EMURX_ID_NONE) lk = EMURX_LK_NO_NS;
    if (ns != EMURX_ID_NONE) r.ns = ns;
    const bool client_kind = ns_ok && key != kNsLevel && key != kNoClient;
    if (client_kind && cid != EMURX_ID_NONE) r.cl = cid;
    set_lk(r, lk);
    // transport: the client's TransportCtx decides (plugin_transport.go:109-114, :73-80)
    const bool trans = key == kMac && (cb == EMURX_CB_TCP || cb == EMURX_CB_UDP) && lk == EMURX_LK_CLIENT;
    if (trans) r.flow = EMURX_FLOW_NO_CTX;
    if (T.ft_on && any_lane(trans) && trans && (cpl & EMURX_CPL_CTX)) r.flow = flow(cid);
}

// GetNs + the callback's client rule against the tables (both bucket reads in flight together)
template <class Flow>
__device__ __forceinline__ void resolve(const emurx_dev_tables& T, Rec& r, const LKey& k, Flow flow) {
    const Probe p = probe_issue(T, r, k);
    Bucket ce{};
    if (p.ctab) ce = ld_bucket(p.ctab, p.cbk);
#if EMURX_FLATRES == 2
    // hybrid: a wave whose lanes share one key kind takes the switch without divergence
    if (__ballot(k.key != (uint32_t)__builtin_amdgcn_readfirstlane((int)k.key)) == 0)
        resolve_done(T, r, k, p, ce, flow);
    else
        resolve_done_flat(T, r, k, p, ce, flow);
#elif EMURX_FLATRES
    resolve_done_flat(T, r, k, p, ce, flow);
#else
    resolve_done(T, r, k, p, ce, flow);
#endif
}

// parse state -> Namespace / Client ids, lookup outcome, flow decision (replicated tables:
// the frame's bytes are at hand, the flow tuple is read only when a flow probe runs)
template <class S>
__device__ __forceinline__ void classify(const S& s, uint32_t len, const emurx_dev_tables& T, Rec& r) {
    if (r.status != EMURX_ST_OK) return;
    const LKey k = make_key(s, len, r);
    resolve(T, r, k, [&](uint32_t cid) { return flow_probe(T, get_tuple(s, len, r), cid); });
}

// ---- partitioned path: the lookup record (include/emu_rx.h emurx_lookup_rec) -----------
// Everything the owner needs to finish the frame: a 32-byte head, and for two classes a tail
// of 16-byte units in the region's tail shards (emu_rx.h).  Head words:
//   w0  source frame index (the source rank is the region the record arrives in)
//   w1  the CTunnelKey VLAN words, 14 bits each (vlan_code): TPID 0x8100 / 0x88A8 / none + VID
//   w2  vport | l3 << 8 | next_hdr << 24          w3  l4 | l7 << 16
//   w4  l7_len | proto << 16 (4 bits, 15 = none) | status << 20 (5 bits) | RTALERT << 25 |
//       v6 << 26 | mc6 << 27 | key << 28 (3 bits) | tuple << 31  (the parse's own flags bit is
//       RTALERT alone)
//   w5  destination MAC bytes 0..3                w6  bytes 4..5 | hi << 16
//   w7  (x) kMac: key bytes 0..3 (hi = bytes 4..5; the destination MAC unless DHCP's chaddr);
//       kIp4: the address; kIp6 / kEui and tuple records: the first tail unit (EMURX_TAIL_NONE
//       when it did not fit)
// kIp6 / kEui (ICMPv6 echo: L7 = L7Len = 0, parser.go:684-717): the client-table hash of the
// key in place of l7 (bits 0..15) and l7_len (16..31), so the owner issues the client probe
// with the Namespace probe and the tail load; tail = the IPv6 destination (4 words).
// tuple (tcp / udp, kMac, while some client has a TransportCtx): hi = the TCP flags byte; tail
// = {ports, src, dst, 0} over IPv4, {ports, src[0..2]} {src[3], dst[0..2]} {dst[3], 0, 0, 0}
// over IPv6 (fillv4tuple / fillv6tuple src/emu/plugins/transport/client_ctx.go:720-765; its
// protocol byte is next_hdr).
__device__ __forceinline__ bool lk_transport(uint32_t cb) { return cb == EMURX_CB_TCP || cb == EMURX_CB_UDP; }
__device__ __forceinline__ bool lk_ip6key(uint32_t key) { return key == kIp6 || key == kEui; }
// a CTunnelKey VLAN word (TPID << 16 | VID, parser.go:810) in 14 bits: ParsePacket only takes
// tags with TPID 0x8100 or 0x88A8, and an untagged slot is 0
__device__ __forceinline__ uint32_t vlan_code(uint32_t v) {
    return v == 0 ? 0u : ((((v >> 16) == 0x8100u) ? 1u : 2u) << 12) | (v & 0xfffu);
}
__device__ __forceinline__ uint32_t vlan_word(uint32_t c) {
    const uint32_t t = (c >> 12) & 3u;
    return t == 0 ? 0u : ((t == 1 ? 0x8100u : 0x88A8u) << 16) | (c & 0xfffu);
}
// the MAC of an EUI-64 IPv6 address (ExtractOnlyMac client_ctx.go:314-329) from its words 2, 3
__device__ __forceinline__ uint2 eui_mac(uint32_t w2, uint32_t w3) {
    return make_uint2(((w2 & 0xff) ^ 2) | (((w2 >> 8) & 0xff) << 8) | (((w2 >> 16) & 0xff) << 16) | (((w3 >> 8) & 0xff) << 24),
                      ((w3 >> 16) & 0xff) | ((w3 >> 24) << 8));
}
// tail units of a head (0, 1 or 3), from its w4
__device__ __forceinline__ uint32_t lk_tail_units(uint32_t w4) {
    const uint32_t key = (w4 >> 28) & 7u;
    if (((w4 >> 20) & 31u) != EMURX_ST_OK) return 0;
    if (lk_ip6key(key)) return 1;
    return (w4 >> 31) ? (((w4 >> 26) & 1u) ? 3u : 1u) : 0u;
}
// the record of a frame; `ok`: it reached a callback (the key words are zero otherwise);
// tup_on: tcp / udp records carry their tuple.  Writes the head (two 16-byte stores) and the
// tail (up to three; LDS: the wave's slab, once the parse is done with it); returns the tail's
// units.
template <class S>
__device__ __forceinline__ uint32_t pack_lookup(const S& s, uint32_t len, const Rec& r, uint32_t frame, bool ok,
                                                bool tup_on, uint4* head, uint4* tail) {
    LKey k{};
    Tuple t{};
    bool tr = false;
    if (ok) {
        k = make_key(s, len, r);
        tr = tup_on && lk_transport(r.proto) && k.key == kMac;
        if (tr) t = get_tuple(s, len, r);
    }
    const bool i6 = ok && lk_ip6key(k.key);
    uint32_t l7 = r.l7, l7len = r.l7len, x = k.kw[0], hi = k.kw[1];
    if (i6) {  // the client-table hash of the key (probe_issue's, with the owner's mask applied there)
        const uint32_t tk = emurx_tk_hash(r.vport, r.vlan0, r.vlan1);
        uint32_t h;
        if (k.key == kEui) {
            const uint2 m = eui_mac(k.kw[2], k.kw[3]);
            h = emurx_mac_hash(tk, m.x, m.y);
        } else {
            h = emurx_ip6_hash(tk, k.kw[0], k.kw[1], k.kw[2], k.kw[3]);
        }
        l7 = h & 0xffffu;
        l7len = h >> 16;
        tail[0] = make_uint4(k.kw[0], k.kw[1], k.kw[2], k.kw[3]);
        hi = 0;
    } else if (tr) {
        hi = t.flags;
        if (!t.v6) {
            tail[0] = make_uint4(t.ports, t.a[0], t.d[0], 0);
        } else {
            tail[0] = make_uint4(t.ports, t.a[0], t.a[1], t.a[2]);
            tail[1] = make_uint4(t.a[3], t.d[0], t.d[1], t.d[2]);
            tail[2] = make_uint4(t.d[3], 0, 0, 0);
        }
    } else if (k.key != kMac) {
        hi = 0;
        if (k.key != kIp4) x = 0;
    }
    const uint32_t w4 = l7len | (min(r.proto, 15u) << 16) | (r.status << 20) | ((r.flags & EMURX_FLAG_RTALERT) << 25) |
                        (t.v6 << 26) | (k.mc6 << 27) | (k.key << 28) | ((uint32_t)tr << 31);
    head[0] = make_uint4(frame, vlan_code(r.vlan0) | (vlan_code(r.vlan1) << 14), r.vport | (r.l3 << 8) | (r.nh << 24),
                         r.l4 | (l7 << 16));
    head[1] = make_uint4(w4, k.dlo, k.dhi | (hi << 16), x);
    return i6 ? 1u : tr ? (t.v6 ? 3u : 1u) : 0u;
}
// the owner's view of a head: the parsed record (ns / client unset) and the lookup key (for
// kIp6 / kEui: its client-table hash in kw[0], the address comes with the tail)
__device__ __forceinline__ LKey unpack_lookup(const uint32_t w[8], Rec& r, uint32_t& chash) {
    r.ns = EMURX_ID_NONE;
    r.cl = EMURX_ID_NONE;
    r.vlan0 = vlan_word(w[1] & 0x3fffu);
    r.vlan1 = vlan_word((w[1] >> 14) & 0x3fffu);
    r.vport = w[2] & 0xffu;
    r.l3 = (w[2] >> 8) & 0xffffu;
    r.nh = w[2] >> 24;
    r.l4 = w[3] & 0xffffu;
    r.l7 = w[3] >> 16;
    r.l7len = w[4] & 0xffffu;
    const uint32_t p4 = (w[4] >> 16) & 15u;
    r.proto = p4 == 15u ? (uint32_t)EMURX_CB_NONE : p4;
    r.status = (w[4] >> 20) & 31u;
    r.flags = (w[4] >> 25) & 1u;
    r.dlen = 0;
    r.flow = EMURX_FLOW_NONE;
    LKey k;
    k.dlo = w[5];
    k.dhi = w[6] & 0xffffu;
    k.key = (w[4] >> 28) & 7u;
    k.mc6 = (w[4] >> 27) & 1u;
    chash = 0;
    k.kw[2] = k.kw[3] = 0;
    if (lk_ip6key(k.key)) {
        chash = r.l7 | (r.l7len << 16);
        r.l7 = r.l7len = 0;  // ICMPv6 leaves both unset
        k.kw[0] = k.kw[1] = 0;
    } else if (w[4] >> 31) {  // tuple record: the key is the destination MAC
        k.kw[0] = k.dlo;
        k.kw[1] = k.dhi;
    } else {
        k.kw[0] = w[7];
        k.kw[1] = w[6] >> 16;
    }
    return k;
}
// the c5tuplekey of a tuple head from its tail units
__device__ __forceinline__ Tuple tail_tuple(const uint32_t w[8], uint4 t0, uint4 t1, uint4 t2) {
    Tuple t{};
    t.v6 = (w[4] >> 26) & 1u;
    t.flags = (w[6] >> 16) & 0xffu;
    t.proto = w[2] >> 24;  // IPv4: the header's protocol field; IPv6: ParserPacketState.NextHeader
    t.ports = t0.x;
    if (!t.v6) {
        t.a[0] = t0.y;
        t.d[0] = t0.z;
    } else {
        t.a[0] = t0.y; t.a[1] = t0.z; t.a[2] = t0.w; t.a[3] = t1.x;
        t.d[0] = t1.y; t.d[1] = t1.z; t.d[2] = t1.w; t.d[3] = t2.x;
    }
    return t;
}

}  // namespace emurx
