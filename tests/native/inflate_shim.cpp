// Test shim: the device inflate core (svt_inflate.h) compiled for the host, checked against zlib
// by tests/test_inflate_core.py.
#include "svt_inflate.h"
extern "C" int inf_host(const uint8_t *in, uint32_t clen, uint8_t *out, uint32_t ulen, uint32_t skip) {
    static uint16_t tabs[3 * IF_FAST]; static InfSlow S;
    InfFast F(tabs + 1, 3);   // a strided view, as on the device
    return inf_block(reinterpret_cast<const InfV4 *>(in - skip), skip, clen, out, ulen, F, S);
}
