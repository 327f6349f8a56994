// Data-block encoder of the SSTable build, gfx950.
//
// Reference: SSTableBuilder.add / finish_block (src/sstable.py:224-268) packing records
// (record.py:66-72: i32 key_size ‖ key ‖ i32 value_size ‖ value, key_size = len(key) in
// CHARACTERS, record.py:24) into DataBlocks (blocks.py:33-37: records ‖ u16 offset per record ‖
// u16 count).  The host plans the blocks (the greedy DataBlockBuilder rule, blocks.py:78-95);
// this kernel does the byte work: one workgroup per block assembles it in LDS from the packed
// key / value spans (one lane per record, aligned 16-byte chunk reads) and writes it out whole
// with 16-byte stores.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

constexpr uint32_t kMaxBlockData = 65536;                                 // u16 offsets (blocks.py:34)
constexpr uint32_t kMaxBlockBytes = kMaxBlockData + 2 * (kMaxBlockData / 8) + 2;  // + offsets + count
constexpr uint32_t kEncodeLds = ((kMaxBlockBytes + 15) & ~15u) + 32;  // + over-read pad of the store

__device__ __forceinline__ void lds_put_u32(uint8_t* p, uint32_t v) {
    p[0] = uint8_t(v);
    p[1] = uint8_t(v >> 8);
    p[2] = uint8_t(v >> 16);
    p[3] = uint8_t(v >> 24);
}

// Bytes [s, e) of src into dst (LDS), read as aligned 16-byte chunks; returns the number of
// UTF-8 characters (bytes that are not 10xxxxxx continuation bytes) when `count`.
__device__ __forceinline__ uint32_t copy_span(const uint8_t* __restrict__ src, uint64_t s, uint64_t e, uint8_t* dst,
                                              bool count) {
    uint32_t chars = 0;
    for (uint64_t a = s & ~uint64_t(15); a < e; a += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + a);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t pos = a + j;
            if (pos >= s && pos < e) {
                const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                dst[pos - s] = uint8_t(c);
                if (count) chars += (c & 0xC0u) != 0x80u;
            }
        }
    }
    return chars;
}

// Block b holds records [block_first[b], block_first[b+1]) and lands at out + block_out[b].
// Key i is keys[ko[i], ko[i+1]), value i is vals[vo[i], vo[i+1]).  A block whose bytes exceed
// kMaxBlockBytes is not written and counts in *err.
__global__ void __launch_bounds__(512) k_encode_blocks(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ ko,
                                                       const uint8_t* __restrict__ vals, const uint64_t* __restrict__ vo,
                                                       const uint64_t* __restrict__ block_first,
                                                       const uint64_t* __restrict__ block_out, uint8_t* __restrict__ out,
                                                       unsigned int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t blk[];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t b = blockIdx.x;
    const uint64_t r0 = block_first[b], r1 = block_first[b + 1];
    const uint32_t cnt = uint32_t(r1 - r0);
    const uint64_t kbase = ko[r0], vbase = vo[r0];
    const uint64_t data_len = (ko[r1] - kbase) + (vo[r1] - vbase) + 8 * uint64_t(cnt);
    const uint64_t total = data_len + 2 * uint64_t(cnt) + 2;
    if (data_len > kMaxBlockData || total > kMaxBlockBytes) {
        if (tid == 0) atomicAdd(err, 1u);
        return;
    }
    // records: one lane per record (offset loads coalesced across the wave); its key and value
    // bytes are read as aligned 16-byte chunks (each holds >= 1 byte of the span, so reads stay
    // on the span's pages) and placed byte by byte in the LDS block
    for (uint32_t i = tid; i < cnt; i += nt) {
        const uint64_t r = r0 + i;
        const uint64_t ks = ko[r], ke = ko[r + 1], vs = vo[r], ve = vo[r + 1];
        const uint32_t roff = uint32_t((ks - kbase) + (vs - vbase) + 8 * uint64_t(i));
        const uint32_t klen = uint32_t(ke - ks), vlen = uint32_t(ve - vs);
        uint8_t* rec = blk + roff;
        const uint32_t chars = copy_span(keys, ks, ke, rec + 4, true);  // UTF-8 characters
        copy_span(vals, vs, ve, rec + 8 + klen, false);
        lds_put_u32(rec, chars);            // record.py:24,56 (len of the str)
        lds_put_u32(rec + 4 + klen, vlen);  // record.py:60
        blk[data_len + 2 * i] = uint8_t(roff);  // blocks.py:34 u16 offset
        blk[data_len + 2 * i + 1] = uint8_t(roff >> 8);
    }
    if (tid == 0) {  // blocks.py:35 u16 number of records
        blk[data_len + 2 * cnt] = uint8_t(cnt);
        blk[data_len + 2 * cnt + 1] = uint8_t(cnt >> 8);
    }
    __syncthreads();
    // out: bytes up to the first 16-byte boundary, then 16-byte stores (each built from five
    // aligned LDS dwords), then the tail bytes
    uint8_t* dst = out + block_out[b];
    const uint32_t head = uint32_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
    const uint32_t h = uint32_t(min<uint64_t>(head, total));
    const uint32_t nq = uint32_t((total - h) / 16);
    if (tid < h) dst[tid] = blk[tid];
    const uint32_t* bw = reinterpret_cast<const uint32_t*>(blk);
    const uint32_t sh = h & 3;
    for (uint32_t q = tid; q < nq; q += nt) {
        const uint32_t o = h + 16 * q, w = o >> 2;
        const uint32_t d0 = bw[w], d1 = bw[w + 1], d2 = bw[w + 2], d3 = bw[w + 3], d4 = bw[w + 4];
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
        *reinterpret_cast<uint4*>(dst + o) = v;
    }
    for (uint32_t t = h + 16 * nq + tid; t < total; t += nt) dst[t] = blk[t];
}

}  // namespace pbf
