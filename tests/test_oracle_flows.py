"""The oracle's transport flow tables: the Go map semantics the device tables mirror
(addFlow refuses duplicates, removeFlow of an absent key fails, a client's removal takes its
flows and listeners, src/emu/plugins/transport/client_ctx.go:579-651)."""
from emurx import abi


def test_flow_table_semantics(oracle_built):
    import pyoracle
    o = pyoracle.Oracle()
    key = bytes(12)
    assert o.ns_add(key, 0, abi.PLUG_ALL) == 0
    mac = bytes([2, 0, 0, 0, 0, 1])
    assert o.client_add(0, 5, mac, bytes([10, 0, 0, 1]), None, None, abi.PLUG_ALL) == 0
    t4, t6 = bytes(range(13)), bytes(range(37))
    assert o.flow_add(5, t4, 7) == 0 and o.flow_add(5, t4, 8) == abi.EMURX_EEXIST
    assert o.flow_add(5, t6, 9) == 0 and o.flow_add(5, bytes(12), 1) == abi.EMURX_EINVAL
    assert o.flow_add(6, t4, 1) == abi.EMURX_ENOENT
    assert o.flow_add(5, bytes(13), abi.FLOW_ID_MAX + 1) == abi.EMURX_EINVAL
    assert o.server_add(5, 80, 6) == 0 and o.server_add(5, 80, 6) == abi.EMURX_EEXIST
    assert o.server_add(5, 80, 1) == abi.EMURX_EINVAL
    assert o.flow_remove(5, t4) == 0 and o.flow_remove(5, t4) == abi.EMURX_ENOENT
    assert o.client_remove(0, mac) == 0
    assert o.client_add(0, 5, mac, None, None, None, abi.PLUG_ALL) == 0
    assert o.flow_remove(5, t6) == abi.EMURX_ENOENT and o.server_remove(5, 80, 6) == abi.EMURX_ENOENT
