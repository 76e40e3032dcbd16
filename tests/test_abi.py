"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/gsim.h declares, validates like the reference, and refuses to
run without a device (there is no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, gpu_available
from gsim import _abi
from gsim.engine import Engine, random_regular
from gsim.params import PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams

HEADER = os.path.join(REPO, "include", "gsim.h")
HEADERS = [HEADER, os.path.join(REPO, "include", "gsim_wire.h")]


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsim_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    fns = declared_functions()
    for must in ["gsim_create", "gsim_destroy", "gsim_load_graph", "gsim_refresh_scores", "gsim_read_scores",
                 "gsim_set_topic_params", "gsim_set_app_score", "gsim_set_ip_whitelist", "gsim_last_error"]:
        assert must in fns


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_signatures_cover_header():
    declared = set(declared_functions())
    bound = {name for name, _, _ in _abi.SIGNATURES}
    assert declared == bound


def test_struct_layout_matches_c(tmp_path):
    """Compile a probe against gsim.h and compare sizeof/offsetof with ctypes."""
    import subprocess
    structs = {"gsim_topic_score_params": _abi.CTopicScoreParams, "gsim_peer_score_params": _abi.CPeerScoreParams,
               "gsim_thresholds": _abi.CThresholds, "gsim_gossipsub_params": _abi.CGossipSubParams,
               "gsim_msg_config": _abi.CMsgConfig, "gsim_msg": _abi.CMsg, "gsim_bytes": _abi.CBytes,
               "gsim_wire_sub": _abi.CWireSub, "gsim_wire_ihave": _abi.CWireIHave, "gsim_wire_iwant": _abi.CWireIWant,
               "gsim_wire_graft": _abi.CWireGraft, "gsim_wire_px": _abi.CWirePx, "gsim_wire_prune": _abi.CWirePrune,
               "gsim_wire_rpc": _abi.CWireRpc, "gsim_wire_names": _abi.CWireNames}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "gsim.h"', '#include "gsim_wire.h"',
             "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_random_regular_generator_is_simple_and_regular():
    net = random_regular(2000, 32, seed=1)
    deg = np.diff(net.row_ptr.astype(np.int64))
    assert (deg == 32).all()
    owner = net.owner()
    assert not (owner == net.col).any()                    # no self loops
    for i in range(0, 2000, 97):                           # rows sorted, no duplicates
        row = net.col[net.row_ptr[i]:net.row_ptr[i + 1]]
        assert (np.diff(row.astype(np.int64)) > 0).all()
    rev = net.rev()
    assert (net.col[rev] == owner).all()                   # symmetric
    assert (net.outbound + net.outbound[rev] == 1).all()   # exactly one initiator per connection
    again = random_regular(2000, 32, seed=1)
    assert (again.col == net.col).all() and (again.outbound == net.outbound).all()


def _params():
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=0.5)
    return PeerScoreParams(AppSpecificScore=lambda p: 0.0, DecayInterval=Second, DecayToZero=0.01,
                           Topics={"t": tp})


def test_create_validates_before_touching_device():
    p = _params()
    p.DecayToZero = 2.0
    with pytest.raises(ValueError, match="DecayToZero"):
        Engine(p, PeerScoreThresholds())
    with pytest.raises(ValueError, match="gossip threshold"):
        Engine(_params(), PeerScoreThresholds(GossipThreshold=1))


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_create_without_device_fails_loudly():
    from gsim.engine import GsimError
    with pytest.raises(GsimError, match="no HIP device"):
        Engine(_params(), PeerScoreThresholds())


def test_every_field_has_a_host_dtype():
    """Each GSIM_F_* view the header declares can be read and written from
    the host mirror (dtype and shape known)."""
    import re
    from gsim import engine
    hdr = open(os.path.join(REPO, "include", "gsim.h")).read()
    body = hdr[hdr.index("GSIM_F_FIRST = 0"):hdr.index("GSIM_F__COUNT")]
    n = len(re.findall(r"^\s*GSIM_F_\w+", body, re.M))
    assert set(range(n)) <= set(engine._FIELD_DTYPES)
