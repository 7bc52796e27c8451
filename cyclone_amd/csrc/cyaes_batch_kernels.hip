// cyaes_batch_kernels.hip -- the batching adapter's device-side gather and
// scatter (include/cyaes_batch.h, cyaes_batcher.cpp).
//
// A batch is a list of request descriptors (BatchDesc, cyaes_internal.h).
// Each names its input and output by DEVICE address: host memory the caller
// registered as a packet pool (hipHostRegister, mapped), or the batcher's own
// pinned bounce buffer for requests outside every pool.  The GPU moves the
// bytes itself over PCIe -- one wave per request, 1 KiB (dwordx4) contiguous
// per wave instruction -- so the host copies nothing:
//   k_batch_gather : input -> the batch's HBM stage, building RELAY_FORWARD
//                    packets for SEAL on the way (relay_local.cpp:189-201:
//                    BE u16 size and id, RelayForwardMsg{id, size} in host
//                    order, the chunk, 0xCE padding to 16, cye_packet.cpp:102),
//                    and writes the ragged kernels' (offset, bytes, key) lists;
//   (k_encrypt_quad / k_encrypt / k_decrypt_ragged run on the stage in HBM;)
//   k_batch_scatter: stage -> outputs: the sealed packet (SEAL), the payload
//                    decrypted in place behind its header, whose bytes are
//                    written back unchanged (OPEN, relay_server.cpp:329), or the
//                    CBC output (ENCRYPT/DECRYPT).
#include <algorithm>

#include "cyaes_internal.h"
#include "cyaes_relay.h"

namespace cyaes {
namespace {

constexpr uint32_t kHead = CYAES_RELAY_HEADSIZE;          // Packet head: BE u16 size, BE u16 id (cye_packet.h:6-25)
constexpr uint32_t kPayload = CYAES_RELAY_PAYLOAD_OFFSET;  // head + RelayForwardMsg{int32 id, int32 size}
constexpr uint32_t kForwardId = CYAES_RELAY_FORWARD;       // relay_protocol.h:9-14
constexpr uint8_t kPad = CYAES_RELAY_PAD;                  // Packet::_resize fill (cye_packet.cpp:102)

// 16 B at a 4-byte-aligned address: still one global_load/store_dwordx4.
struct __attribute__((aligned(4))) Blk4 {
    uint32_t x, y, z, w;
};

// dst[0, n) = src[0, n), one wave.  When both ends are 4-B aligned: 16 B per
// lane (dwordx4 at 4-B alignment), then the last n % 16 bytes as dwords; else
// bytes.  Each round issues all its loads before its stores (4 KiB per wave),
// so a relay packet costs one or two PCIe round trips.  The callers place the
// HBM stage so that the host end of every copy keeps its own alignment (a
// whole relay packet moves, header included), and only the HBM end of a copy
// is off 16 B.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane) {
    const uintptr_t a = (uintptr_t)dst | (uintptr_t)src;
    uint32_t body = 0;
    if ((a & 3u) == 0) {
        body = n & ~15u;
        for (uint32_t o0 = 0; o0 < body; o0 += 4096) {
            Blk4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t o = o0 + 1024 * k + 16 * lane;
                if (o < body) v[k] = *reinterpret_cast<const Blk4*>(src + o);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t o = o0 + 1024 * k + 16 * lane;
                if (o < body) *reinterpret_cast<Blk4*>(dst + o) = v[k];
            }
        }
        const uint32_t o = body + 4 * lane;  // at most 3 dwords
        if (o + 4 <= n) *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(src + o);
        body = n & ~3u;
    }
    for (uint32_t o = body + lane; o < n; o += 64) dst[o] = src[o];
}

__device__ __forceinline__ bool is_relay(uint32_t op) { return op >= kOpRelaySeal; }

// Gather of request i: input -> stage, and the ragged kernels' list entry i.
// Requests [0, ne) are the encrypt list (ENCRYPT, SEAL), [ne, n) the decrypt
// list (DECRYPT, OPEN); the decrypt kernel gets the lists from ne.
__device__ __forceinline__ void gather_one(const BatchDesc& d, uint32_t i, uint8_t* __restrict__ stage,
                                           uint64_t* __restrict__ offs, uint32_t* __restrict__ nbytes,
                                           uint32_t* __restrict__ kidx, uint32_t lane) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
    uint8_t* s = stage + d.stage;
    if (lane == 0) {
        offs[i] = is_relay(d.op) ? d.stage + 16 : d.stage;  // relay payload 16-B aligned at stage + 16
        nbytes[i] = d.crypt;
        kidx[i] = d.key;
    }
    switch (d.op) {
        case kOpEncrypt:
        case kOpDecrypt:
            wave_copy(s, src, d.size, lane);
            break;
        case kOpRelaySeal: {  // packet at stage + 4, so its payload (offset 12) is at stage + 16
            uint8_t* pk = s + kHead;
            if (lane == 0) {
                const uint32_t psize = 8 + d.crypt;
                pk[0] = (uint8_t)(psize >> 8);
                pk[1] = (uint8_t)psize;
                pk[2] = (uint8_t)(kForwardId >> 8);
                pk[3] = (uint8_t)kForwardId;
                *reinterpret_cast<int32_t*>(pk + 4) = d.conn;          // RelayForwardMsg::id
                *reinterpret_cast<int32_t*>(pk + 8) = (int32_t)d.size; // RelayForwardMsg::size
            }
            wave_copy(pk + kPayload, src, d.size, lane);
            for (uint32_t o = d.size + lane; o < d.crypt; o += 64) pk[kPayload + o] = kPad;
            break;
        }
        case kOpRelayOpen:  // the whole packet at stage + 4 (payload at stage + 16): the host
                            // end keeps the packet's alignment
            wave_copy(s + kHead, src, kPayload + d.crypt, lane);
            break;
    }
}

__device__ __forceinline__ void scatter_one(const BatchDesc& d, const uint8_t* __restrict__ stage, uint32_t lane) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(d.dst);
    const uint8_t* s = stage + d.stage;
    switch (d.op) {
        case kOpEncrypt:
        case kOpDecrypt:
            wave_copy(dst, s, d.size, lane);
            break;
        case kOpRelaySeal:  // the whole packet: header, RelayForwardMsg, ciphertext
            wave_copy(dst, s + kHead, kPayload + d.crypt, lane);
            break;
        case kOpRelayOpen:  // plaintext back behind the header, in place; the header's 12
                            // bytes are written back unchanged so that the host end is
                            // the packet's own alignment (the gather read them)
            wave_copy(dst, s + kHead, kPayload + d.crypt, lane);
            break;
    }
}

// One launch moves both PCIe directions: the scatter of batch k (its outputs,
// stage -> host pools) and the gather of batch k+1 (inputs, host pools ->
// stage), so the batcher's single in-order pipeline stream keeps H2D and D2H
// busy at once.  The waves split between the two lists in proportion to
// their request counts; one wave per request, grid-stride.
__global__ void k_batch_move(BatchMove m) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    const uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t tot = (uint64_t)m.gn + m.sn;
    const uint32_t gw = m.sn == 0 ? nw : m.gn == 0 ? 0 : (uint32_t)max<uint64_t>(1, min<uint64_t>(nw - 1, nw * m.gn / tot));
    if (w < gw) {
        for (uint32_t i = w; i < m.gn; i += gw) gather_one(m.gdesc[i], i, m.gstage, m.offs, m.nbytes, m.kidx, lane);
    } else {
        const uint32_t sw = nw - gw;
        for (uint32_t i = w - gw; i < m.sn; i += sw) scatter_one(m.sdesc[i], m.sstage, lane);
    }
}

}  // namespace

hipError_t launch_batch_move(const BatchMove& m, int max_waves, hipStream_t stream) {
    const uint64_t n = (uint64_t)m.gn + m.sn;
    if (n == 0) return hipSuccess;
    const uint32_t waves = (uint32_t)std::min<uint64_t>(n, (uint64_t)std::max(2, max_waves));
    hipLaunchKernelGGL(k_batch_move, dim3((waves + 3) / 4), dim3(256), 0, stream, m);
    return hipGetLastError();
}

}  // namespace cyaes
