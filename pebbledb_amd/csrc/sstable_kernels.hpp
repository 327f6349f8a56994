// Data-block encoder of the SSTable build, gfx950.
//
// Reference: SSTableBuilder.add / finish_block (src/sstable.py:224-268) packing records
// (record.py:66-72: i32 key_size ‖ key ‖ i32 value_size ‖ value, key_size = len(key) in
// CHARACTERS, record.py:24) into DataBlocks (blocks.py:33-37: records ‖ u16 offset per record ‖
// u16 count).  The host plans the blocks (the greedy DataBlockBuilder rule, blocks.py:78-95);
// this kernel does the byte work: one workgroup per block assembles it in LDS from the packed
// key / value spans (wave-cooperative, byte-coalesced reads) and writes it out whole.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

constexpr uint32_t kMaxBlockData = 65536;                                 // u16 offsets (blocks.py:34)
constexpr uint32_t kMaxBlockBytes = kMaxBlockData + 2 * (kMaxBlockData / 8) + 2;  // + offsets + count
constexpr uint32_t kEncodeLds = (kMaxBlockBytes + 15) & ~15u;

__device__ __forceinline__ void lds_put_u32(uint8_t* p, uint32_t v) {
    p[0] = uint8_t(v);
    p[1] = uint8_t(v >> 8);
    p[2] = uint8_t(v >> 16);
    p[3] = uint8_t(v >> 24);
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
    const uint32_t lane = tid & 63, wave = tid >> 6, nwaves = nt >> 6;
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
    // records: one wave per record, 64 bytes per step
    for (uint32_t i = wave; i < cnt; i += nwaves) {
        const uint64_t r = r0 + i;
        const uint64_t ks = ko[r], ke = ko[r + 1], vs = vo[r], ve = vo[r + 1];
        const uint32_t roff = uint32_t((ks - kbase) + (vs - vbase) + 8 * uint64_t(i));
        const uint32_t klen = uint32_t(ke - ks), vlen = uint32_t(ve - vs);
        uint8_t* rec = blk + roff;
        uint32_t chars = 0;  // UTF-8 characters = bytes that are not continuation bytes
        for (uint32_t t0 = 0; t0 < klen; t0 += 64) {
            const uint32_t t = t0 + lane;
            uint8_t c = 0;
            if (t < klen) {
                c = keys[ks + t];
                rec[4 + t] = c;
            }
            chars += uint32_t(__popcll(__ballot(t < klen && (c & 0xC0) != 0x80)));
        }
        for (uint32_t t = lane; t < vlen; t += 64) rec[8 + klen + t] = vals[vs + t];
        if (lane == 0) {
            lds_put_u32(rec, chars);              // record.py:24,56 (len of the str)
            lds_put_u32(rec + 4 + klen, vlen);    // record.py:60
            blk[data_len + 2 * i] = uint8_t(roff);  // blocks.py:34 u16 offset
            blk[data_len + 2 * i + 1] = uint8_t(roff >> 8);
        }
    }
    if (tid == 0) {  // blocks.py:35 u16 number of records
        blk[data_len + 2 * cnt] = uint8_t(cnt);
        blk[data_len + 2 * cnt + 1] = uint8_t(cnt >> 8);
    }
    __syncthreads();
    uint8_t* dst = out + block_out[b];
    for (uint32_t t = tid; t < total; t += nt) dst[t] = blk[t];
}

}  // namespace pbf
