"""Single-process multi-GPU front end (include/cyaes_mgpu.h): RCCL key
broadcast + sharded uniform batches, against the oracle.  The GPU box has one
device, so the clique has one member here; the shard / key-offset logic is
exercised by giving that device a shard that does not start at payload 0."""
import pytest

import cyclone_amd as ca
import oracle

pytestmark = pytest.mark.gpu


def test_broadcast_and_sharded_batches_match_oracle():
    import torch
    mg = ca.MultiGpu([0])
    assert mg.ndev == 1
    nkeys, ppk, pb = 16, 8, 1472
    keys = [oracle.session_key(s) for s in range(nkeys)]
    mg.broadcast_keys(b"".join(keys), root=0)
    total = nkeys * ppk
    for first, count in [(0, total), (3 * ppk, 5 * ppk), (ca.mgpu_shard(total, 4, 3, ppk))]:
        plain = oracle.synthetic(first, count, pb)
        d_in = torch.from_numpy(plain).cuda()
        d_ct = torch.empty_like(d_in)
        d_rt = torch.empty_like(d_in)
        mg.encrypt_uniform([d_in], [d_ct], [count], [first], pb, ppk)
        mg.decrypt_uniform([d_ct], [d_rt], [count], [first], pb, ppk)
        ct = d_ct.cpu().numpy()
        for p in range(count):
            k = keys[(first + p) // ppk]
            want = oracle.Rijndael(k).encrypt(bytearray(plain[p * pb:(p + 1) * pb].tobytes()))
            assert ct[p * pb:(p + 1) * pb].tobytes() == bytes(want)
        assert torch.equal(d_rt, d_in)
    with pytest.raises(ca.CyaesError) as e:  # shard not on a session boundary
        mg.encrypt_uniform([d_in], [d_ct], [1], [1], pb, ppk)
    assert e.value.status == ca.CYAES_EINVAL
    with pytest.raises(ca.CyaesError) as e:  # beyond the broadcast key table
        mg.encrypt_uniform([d_in], [d_ct], [ppk + 1], [total - ppk], pb, ppk)
    assert e.value.status == ca.CYAES_ERANGE
    mg.close()
