// GPU decode of serialized tf.train.Example records (TF's ParseExample on the
// reference's input path, PS:79-133 / HVD:79-133), the streamed-epoch half of the input pipeline.
//
// The host loader (csrc/io/hfm_io.cpp, raw mode) only frames TFRecords and checks their length
// CRCs and ships each batch as the records' bytes back to back + B + 1 offsets (crc mode: each
// record followed by its data CRC, verified here -- the host does no per-byte work at all);
// this kernel writes the fixed-schema features straight into a device ring slot:
//   label f32 [B], ids int32 [B, F] (checked against [0, V) and int32), values f32 [B, F].
// Schema (any field / map-entry order, unknown fields skipped):
//   Example { 1: Features { 1: repeated MapEntry { 1: key, 2: Feature { 2: FloatList | 3: Int64List } } } }
//   FloatList / Int64List { 1: packed (LEN) or repeated (fixed32 / varint) values }
// One wave per record: the record is copied into the wave's slice of LDS by all 64 lanes, the
// message structure is walked wave-uniformly from LDS, and the packed ids are decoded 64 bytes at
// a time -- a ballot of the varint terminator bits gives every terminator lane its id index and
// its varint's first byte, so each id is assembled by one lane.
// Errors never fault: a record that does not match the schema gets zero ids / values and sets
// err[0] bit 0, an id outside [0, V) or int32 is written as 0 and sets bit 1, a data CRC mismatch
// (crc mode) zeroes the row and sets bit 2; err[1] holds the smallest bad record index of the
// batch (the host reports it).
#include "common.h"

namespace {

// ---- TFRecord data CRC (crc mode): masked CRC32C of the payload, checked here instead of on the
// host (the host's serial crc32 chain was ~57 ns of its ~66 ns per record).  Tables are built at
// compile time.  Slice-by-8 over 8-byte steps; 8 lanes each take one of 8 equal segments (the
// message is conceptually front-padded with zero bytes to 8 * seg: leading zeros leave a CRC
// register of 0 unchanged) and the partial CRCs are combined in a shuffle tree, multiplying by
// x^(8 seg), x^(16 seg), x^(32 seg) mod P; the initial register ~0 is folded in by inverting the
// first 4 message bytes (a 32-bit reflected CRC depends on state ^ first word only).
constexpr uint32_t CRC_POLY = 0x82F63B78u;    // CRC32C, reflected
constexpr uint32_t crc_x1(uint32_t b) { return (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1; }   // b * x
__host__ __device__ constexpr uint32_t crc_mulmod(uint32_t a, uint32_t b) {                    // a * b mod P
  uint32_t p = 0;
  for (int k = 0; k < 32; ++k) {
    if (a & (0x80000000u >> k)) p ^= b;
    b = crc_x1(b);
  }
  return p;
}
struct CrcTabs {
  uint32_t t[8][256];
};
constexpr CrcTabs make_crc_tabs() {
  CrcTabs T{};
  for (int i = 0; i < 256; ++i) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = crc_x1(c);
    T.t[0][i] = c;
  }
  for (int k = 1; k < 8; ++k)
    for (int i = 0; i < 256; ++i) T.t[k][i] = (T.t[k - 1][i] >> 8) ^ T.t[0][T.t[k - 1][i] & 0xFFu];
  return T;
}
constexpr int CRC_SEGS = 128;                 // parallel path: seg = 8 (s + 1) bytes, n <= 8 * 1024
struct CrcOps {
  uint32_t op[CRC_SEGS][3];                   // x^(8 seg), x^(16 seg), x^(32 seg) mod P
};
constexpr CrcOps make_crc_ops() {
  CrcOps O{};
  uint32_t x = 0x80000000u;                   // x^0
  for (int s = 0; s < CRC_SEGS; ++s) {
    for (int k = 0; k < 64; ++k) x = crc_x1(x);
    O.op[s][0] = x;
    O.op[s][1] = crc_mulmod(x, x);
    O.op[s][2] = crc_mulmod(O.op[s][1], O.op[s][1]);
  }
  return O;
}
__constant__ CrcTabs kCrcT = make_crc_tabs();
__constant__ CrcOps kCrcOps = make_crc_ops();

// masked CRC32C of the payload [0, n) of r (valid in lane 0)
template <class R>
__device__ uint32_t payload_crc(const R& r, uint32_t n, int lane) {
  uint32_t v = 0;
  if (n < 64 || n > 8u * 8u * CRC_SEGS) {     // short / very long: one lane, plain byte loop
    if (lane == 0) {
      v = 0xFFFFFFFFu;
      for (uint32_t i = 0; i < n; ++i) v = kCrcT.t[0][(v ^ r.at(i)) & 0xFFu] ^ (v >> 8);
      v = ~v;
    }
  } else {
    const uint32_t seg = ((n + 63u) / 64u) * 8u, z = 8u * seg - n;
    if (lane < 8) {
      const int b1 = (int)((lane + 1) * seg) - (int)z;
      int pos = max((int)(lane * seg) - (int)z, 0);
      auto byte = [&](int i) { return r.at((uint32_t)i) ^ (i < 4 ? 0xFFu : 0u); };
      while (pos < b1 && ((b1 - pos) & 7)) {   // (a lane wholly inside the zero padding: b1 <= 0)
        v = kCrcT.t[0][(v ^ byte(pos)) & 0xFFu] ^ (v >> 8);
        ++pos;
      }
      for (; pos < b1; pos += 8) {
        const uint32_t lo = byte(pos) | (byte(pos + 1) << 8) | (byte(pos + 2) << 16) | (byte(pos + 3) << 24);
        const uint32_t hi = byte(pos + 4) | (byte(pos + 5) << 8) | (byte(pos + 6) << 16) | (byte(pos + 7) << 24);
        v ^= lo;
        v = kCrcT.t[7][v & 0xFFu] ^ kCrcT.t[6][(v >> 8) & 0xFFu] ^ kCrcT.t[5][(v >> 16) & 0xFFu] ^ kCrcT.t[4][v >> 24] ^
            kCrcT.t[3][hi & 0xFFu] ^ kCrcT.t[2][(hi >> 8) & 0xFFu] ^ kCrcT.t[1][(hi >> 16) & 0xFFu] ^ kCrcT.t[0][hi >> 24];
      }
    }
    const uint32_t* op = kCrcOps.op[seg / 8u - 1u];
#pragma unroll
    for (int l = 0; l < 3; ++l) {             // (v_i, v_{i + 2^l}) -> v_i * x^(8 seg 2^l) ^ v_{i + 2^l}
      const uint32_t o = (uint32_t)__shfl_down((int)v, 1 << l, 64);
      if ((lane & ((2 << l) - 1)) == 0 && lane < 8) v = crc_mulmod(op[l], v) ^ o;
    }
    v = ~v;
  }
  return ((v >> 15) | (v << 17)) + 0xa282ead8u;
}

constexpr int DEC_WAVES = 4;          // records per 256-thread workgroup
constexpr int DEC_STAGE = 1024;       // LDS bytes per wave (longer records read the rest from memory)

struct Rec {
  const uint8_t* g;                   // the record in global memory
  const uint8_t* s;                   // its first DEC_STAGE bytes in LDS
  uint32_t n;                         // record length
  __device__ __forceinline__ uint32_t at(uint32_t i) const { return i < DEC_STAGE ? s[i] : g[i]; }
};

// wave-uniform varint at *pos (advances it); false if it runs past `end` or over 10 bytes
__device__ __forceinline__ bool rd_varint(const Rec& r, uint32_t& pos, uint32_t end, uint64_t& v) {
  v = 0;
  for (int sh = 0; sh < 70; sh += 7) {
    if (pos >= end) return false;
    const uint32_t c = r.at(pos++);
    v |= (uint64_t)(c & 0x7Fu) << sh;
    if (!(c & 0x80u)) return true;
  }
  return false;
}

__device__ __forceinline__ bool skip_field(const Rec& r, uint32_t& pos, uint32_t end, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return rd_varint(r, pos, end, v);
    case 1: pos += 8; return pos <= end;
    case 2:
      if (!rd_varint(r, pos, end, v) || v > end - pos) return false;
      pos += (uint32_t)v;
      return true;
    case 5: pos += 4; return pos <= end;
    default: return false;
  }
}

__device__ __forceinline__ float rd_f32(const Rec& r, uint32_t pos) {
  const uint32_t u = r.at(pos) | (r.at(pos + 1) << 8) | (r.at(pos + 2) << 16) | (r.at(pos + 3) << 24);
  return __uint_as_float(u);
}

// FloatList payload [pos, end) -> dst[0, want); false unless exactly `want` values
__device__ bool dec_floats(const Rec& r, uint32_t pos, uint32_t end, float* dst, int want, int lane) {
  int n = 0;
  while (pos < end) {
    uint64_t key;
    if (!rd_varint(r, pos, end, key)) return false;
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f != 1) {
      if (!skip_field(r, pos, end, wt)) return false;
      continue;
    }
    if (wt == 2) {
      uint64_t len;
      if (!rd_varint(r, pos, end, len) || len > end - pos || (len & 3)) return false;
      const int k = (int)(len / 4);
      if (n + k > want) return false;
      for (int i = lane; i < k; i += 64) dst[n + i] = rd_f32(r, pos + 4 * i);
      n += k;
      pos += (uint32_t)len;
    } else if (wt == 5) {
      if (pos + 4 > end || n + 1 > want) return false;
      if (lane == 0) dst[n] = rd_f32(r, pos);
      ++n;
      pos += 4;
    } else {
      return false;
    }
  }
  return n == want;
}

// one decoded id: checked, narrowed, stored (lane-private)
__device__ __forceinline__ void put_id(int32_t* dst, int idx, uint64_t v, int64_t limit, unsigned& bad) {
  const bool ok = v <= 0x7FFFFFFFull && (limit <= 0 || (int64_t)v < limit);
  if (!ok) bad |= 2u;
  dst[idx] = ok ? (int32_t)v : 0;
}

// Int64List payload [pos, end) -> dst[0, want) as int32; false unless exactly `want` values
__device__ bool dec_ids(const Rec& r, uint32_t pos, uint32_t end, int32_t* dst, int want, int64_t limit,
                        int lane, unsigned& bad) {
  int n = 0;
  while (pos < end) {
    uint64_t key;
    if (!rd_varint(r, pos, end, key)) return false;
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f != 1) {
      if (!skip_field(r, pos, end, wt)) return false;
      continue;
    }
    if (wt == 0) {                      // unpacked: one varint
      uint64_t v;
      if (!rd_varint(r, pos, end, v) || n + 1 > want) return false;
      if (lane == 0) put_id(dst, n, v, limit, bad);
      ++n;
      continue;
    }
    if (wt != 2) return false;
    uint64_t len;
    if (!rd_varint(r, pos, end, len) || len > end - pos) return false;
    const uint32_t pe = pos + (uint32_t)len;
    uint32_t start = pos;               // first byte of the varint being read
    for (uint32_t base = pos; base < pe; base += 64) {
      const uint32_t q = base + lane;
      const uint32_t c = q < pe ? r.at(q) : 0x80u;
      const bool term = q < pe && !(c & 0x80u);
      const unsigned long long mask = __ballot(term);
      const unsigned long long below = lane ? (mask & ((1ull << lane) - 1)) : 0ull;
      if (term) {
        const uint32_t s0 = below ? base + (63 - __clzll(below)) + 1 : start;
        const int idx = n + __popcll(below);
        if (q - s0 < 10 && idx < want) {
          uint64_t v = 0;
          for (uint32_t t = s0; t <= q; ++t) v |= (uint64_t)(r.at(t) & 0x7Fu) << (7 * (t - s0));
          put_id(dst, idx, v, limit, bad);
        } else {
          bad |= 1u;
        }
      }
      n += __popcll(mask);
      if (mask) start = base + (63 - __clzll(mask)) + 1;
    }
    if (start != pe) return false;      // a varint ran past the payload
    pos = pe;
  }
  return n == want;
}

__device__ __forceinline__ bool name_is(const Rec& r, uint32_t pos, uint32_t len, const char* s, uint32_t n) {
  if (len != n) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (r.at(pos + i) != (uint32_t)(uint8_t)s[i]) return false;
  return true;
}

__global__ void __launch_bounds__(64 * DEC_WAVES) decode_examples_kernel(
    const uint8_t* __restrict__ raw, const uint32_t* __restrict__ offs, int rows, int F, int64_t limit,
    int32_t* __restrict__ ids, float* __restrict__ vals, float* __restrict__ labels, int* __restrict__ err,
    int crc) {
  __shared__ uint8_t stage[DEC_WAVES][DEC_STAGE];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rec = blockIdx.x * DEC_WAVES + wv;
  if (rec >= rows) return;                                  // (wave-uniform)
  const uint32_t o0 = offs[rec], o1 = offs[rec + 1];
  Rec r{raw + o0, stage[wv], o1 - o0};
  const uint32_t ns = r.n < DEC_STAGE ? r.n : DEC_STAGE;
  for (uint32_t i = lane; i < ns; i += 64) stage[wv][i] = r.g[i];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int32_t* idr = ids + (size_t)rec * F;
  float* vr = vals + (size_t)rec * F;
  unsigned bad = 0;
  int have = 0;
  uint32_t pos = 0;
  uint32_t end = r.n;
  bool ok = true;
  if (crc) {                            // the record's last 4 bytes: its masked data CRC
    if (r.n < 4) {
      ok = false;
    } else {
      end = r.n - 4;
      const uint32_t want = r.at(end) | (r.at(end + 1) << 8) | (r.at(end + 2) << 16) | (r.at(end + 3) << 24);
      const uint32_t got = (uint32_t)__shfl((int)payload_crc(r, end, lane), 0, 64);
      if (got != want) {
        bad |= 4u;
        ok = false;
      }
    }
  }
  while (ok && pos < end) {
    uint64_t key;
    if (!rd_varint(r, pos, end, key)) { ok = false; break; }
    if ((key >> 3) != 1 || (key & 7) != 2) {
      ok = skip_field(r, pos, end, (int)(key & 7));
      continue;
    }
    uint64_t flen;
    if (!rd_varint(r, pos, end, flen) || flen > end - pos) { ok = false; break; }
    uint32_t fp = pos;                                        // Features
    const uint32_t fe = pos + (uint32_t)flen;
    pos = fe;
    while (ok && fp < fe) {
      uint64_t k2;
      if (!rd_varint(r, fp, fe, k2)) { ok = false; break; }
      if ((k2 >> 3) != 1 || (k2 & 7) != 2) {
        ok = skip_field(r, fp, fe, (int)(k2 & 7));
        continue;
      }
      uint64_t l2;
      if (!rd_varint(r, fp, fe, l2) || l2 > fe - fp) { ok = false; break; }
      uint32_t mp = fp;                                       // map entry {1: key, 2: Feature}
      const uint32_t me = fp + (uint32_t)l2;
      fp = me;
      uint32_t npos = 0, nlen = 0, vp = 0, ve = 0;
      bool hn = false, hv = false;
      while (mp < me) {
        uint64_t k3, l3;
        if (!rd_varint(r, mp, me, k3)) { ok = false; break; }
        if ((k3 & 7) != 2) {
          if (!skip_field(r, mp, me, (int)(k3 & 7))) { ok = false; break; }
          continue;
        }
        if (!rd_varint(r, mp, me, l3) || l3 > me - mp) { ok = false; break; }
        if ((k3 >> 3) == 1) { npos = mp; nlen = (uint32_t)l3; hn = true; }
        else if ((k3 >> 3) == 2) { vp = mp; ve = mp + (uint32_t)l3; hv = true; }
        mp += (uint32_t)l3;
      }
      if (!ok || !hn || !hv) continue;
      uint64_t k4, l4;                                        // Feature { oneof 1 / 2 / 3 }
      uint32_t q = vp;
      if (!rd_varint(r, q, ve, k4) || (k4 & 7) != 2 || !rd_varint(r, q, ve, l4) || l4 > ve - q) {
        ok = false;
        break;
      }
      const int kind = (int)(k4 >> 3);
      const uint32_t qe = q + (uint32_t)l4;
      if (kind == 2 && name_is(r, npos, nlen, "label", 5)) {
        ok = dec_floats(r, q, qe, labels + rec, 1, lane);
        have |= 1;
      } else if (kind == 3 && name_is(r, npos, nlen, "ids", 3)) {
        ok = dec_ids(r, q, qe, idr, F, limit, lane, bad);
        have |= 2;
      } else if (kind == 2 && name_is(r, npos, nlen, "values", 6)) {
        ok = dec_floats(r, q, qe, vr, F, lane);
        have |= 4;
      }
    }
  }
  if (!(bad & 4u) && (!ok || have != 7)) bad |= 1u;
  if (bad & 5u) {                       // schema / CRC mismatch: a defined (zero) row, never garbage ids
    for (int f = lane; f < F; f += 64) {
      idr[f] = 0;
      vr[f] = 0.f;
    }
    if (lane == 0) labels[rec] = 0.f;
  }
  // (lanes disagree only on bit 1: the lanes that decoded a bad id)
  const unsigned long long any = __ballot(bad != 0);
  if (any) {
    unsigned allbad = bad;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) allbad |= __shfl_xor(allbad, o, 64);
    if (lane == 0) {
      atomicOr(err, (int)allbad);
      atomicMin(err + 1, rec);
    }
  }
}

}  // namespace

// raw: the batch's record bytes; offs: rows + 1 start offsets (offs[rows] = total bytes).
// err: [2] ints, err[1] initialised to INT_MAX by the caller (the smallest bad record index).
// crc: 1 = every record ends with its 4-byte masked data CRC (the raw loader's verify mode 2),
// checked here (err bit 2 = value 4: mismatch; the row is zeroed)
HFM_API int hfm_decode_examples(const void* raw, const void* offs, int rows, int F, long long limit, void* ids,
                                void* vals, void* labels, void* err, int crc, hipStream_t st) {
  if (rows <= 0) return 0;
  if (F <= 0 || !raw || !offs || !ids || !vals || !labels || !err) return (int)hipErrorInvalidValue;
  const int grid = (rows + DEC_WAVES - 1) / DEC_WAVES;
  hipLaunchKernelGGL(decode_examples_kernel, dim3(grid), dim3(64 * DEC_WAVES), 0, st, (const uint8_t*)raw,
                     (const uint32_t*)offs, rows, F, (int64_t)limit, (int32_t*)ids, (float*)vals, (float*)labels,
                     (int*)err, crc);
  HFM_LAUNCH_CHECK();
}
