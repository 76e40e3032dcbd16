"""The GossipSub wire format through libgsim (include/gsim_wire.h).

Mirrors the reference's protobuf types (pb/rpc.proto:5-57) as dataclasses
with the same field names, so code written against `pb.RPC` reads the same:
`marshal(rpc)` is `rpc.Marshal()`, `size(rpc)` is `rpc.Size()`,
`fragment_rpc(rpc, limit)` is `fragmentRPC` (gossipsub.go:1204-1296; it
returns the fragments encoded).  `heartbeat_rpcs(engine, ...)` reads back the
RPCs the engine's routers sent at a heartbeat, encoded on the device.

Optional fields are absent when None (proto2 presence); an empty bytes value
is present and encoded, as Go encodes a non-nil empty slice.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _abi


class WireError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gsim wire error {code}: {msg}")
        self.code = code


def _b(x) -> Optional[bytes]:
    if x is None:
        return None
    return x.encode() if isinstance(x, str) else bytes(x)


@dataclass
class SubOpts:                   # RPC.SubOpts
    subscribe: Optional[bool] = None
    topicid: Optional[bytes] = None


@dataclass
class Message:                   # Message
    from_: Optional[bytes] = None
    data: Optional[bytes] = None
    seqno: Optional[bytes] = None
    topic: Optional[bytes] = None
    signature: Optional[bytes] = None
    key: Optional[bytes] = None


@dataclass
class ControlIHave:
    topicID: Optional[bytes] = None
    messageIDs: List[bytes] = field(default_factory=list)


@dataclass
class ControlIWant:
    messageIDs: List[bytes] = field(default_factory=list)


@dataclass
class ControlGraft:
    topicID: Optional[bytes] = None


@dataclass
class PeerInfo:
    peerID: Optional[bytes] = None
    signedPeerRecord: Optional[bytes] = None


@dataclass
class ControlPrune:
    topicID: Optional[bytes] = None
    peers: List[PeerInfo] = field(default_factory=list)
    backoff: Optional[int] = None


@dataclass
class ControlMessage:
    ihave: List[ControlIHave] = field(default_factory=list)
    iwant: List[ControlIWant] = field(default_factory=list)
    graft: List[ControlGraft] = field(default_factory=list)
    prune: List[ControlPrune] = field(default_factory=list)


@dataclass
class RPC:
    subscriptions: List[SubOpts] = field(default_factory=list)
    publish: List[Message] = field(default_factory=list)
    control: Optional[ControlMessage] = None


class _Tables:
    """The flat gsim_wire_rpc tables of an RPC (keeps every buffer alive)."""

    def __init__(self, rpc: RPC):
        self._keep = []
        c = rpc.control
        ids: List[bytes] = []
        pxs: List[PeerInfo] = []
        subs = (_abi.CWireSub * max(1, len(rpc.subscriptions)))()
        for k, s in enumerate(rpc.subscriptions):
            subs[k].subscribe = -1 if s.subscribe is None else int(bool(s.subscribe))
            subs[k].topic = self.bytes(s.topicid)
        msgs = (_abi.CWireMsg * max(1, len(rpc.publish)))()
        for k, m in enumerate(rpc.publish):
            msgs[k].from_ = self.bytes(m.from_)
            msgs[k].data = self.bytes(m.data)
            msgs[k].seqno = self.bytes(m.seqno)
            msgs[k].topic = self.bytes(m.topic)
            msgs[k].signature = self.bytes(m.signature)
            msgs[k].key = self.bytes(m.key)
        ihave = (_abi.CWireIHave * max(1, len(c.ihave) if c else 1))()
        iwant = (_abi.CWireIWant * max(1, len(c.iwant) if c else 1))()
        graft = (_abi.CWireGraft * max(1, len(c.graft) if c else 1))()
        prune = (_abi.CWirePrune * max(1, len(c.prune) if c else 1))()
        if c:
            for k, g in enumerate(c.ihave):
                ihave[k].topic = self.bytes(g.topicID)
                ihave[k].id0, ihave[k].nid = len(ids), len(g.messageIDs)
                ids += [_b(x) for x in g.messageIDs]
            for k, g in enumerate(c.iwant):
                iwant[k].id0, iwant[k].nid = len(ids), len(g.messageIDs)
                ids += [_b(x) for x in g.messageIDs]
            for k, g in enumerate(c.graft):
                graft[k].topic = self.bytes(g.topicID)
            for k, p in enumerate(c.prune):
                prune[k].topic = self.bytes(p.topicID)
                prune[k].px0, prune[k].npx = len(pxs), len(p.peers)
                pxs += p.peers
                prune[k].has_backoff = 0 if p.backoff is None else 1
                prune[k].backoff = p.backoff or 0
        idt = (_abi.CBytes * max(1, len(ids)))()
        for k, x in enumerate(ids):
            idt[k] = self.bytes(x)
        pxt = (_abi.CWirePx * max(1, len(pxs)))()
        for k, x in enumerate(pxs):
            pxt[k].peer = self.bytes(x.peerID)
            pxt[k].record = self.bytes(x.signedPeerRecord)
        self._keep += [subs, msgs, ihave, iwant, graft, prune, idt, pxt]
        r = _abi.CWireRpc()
        r.subs, r.nsubs = ctypes.addressof(subs), len(rpc.subscriptions)
        r.msgs, r.nmsgs = ctypes.addressof(msgs), len(rpc.publish)
        r.has_control = 1 if c is not None else 0
        r.ihave, r.nihave = ctypes.addressof(ihave), len(c.ihave) if c else 0
        r.iwant, r.niwant = ctypes.addressof(iwant), len(c.iwant) if c else 0
        r.graft, r.ngraft = ctypes.addressof(graft), len(c.graft) if c else 0
        r.prune, r.nprune = ctypes.addressof(prune), len(c.prune) if c else 0
        r.ids, r.nids = ctypes.addressof(idt), len(ids)
        r.px, r.npx = ctypes.addressof(pxt), len(pxs)
        self.rpc = r

    def bytes(self, x) -> _abi.CBytes:
        x = _b(x)
        if x is None:
            return _abi.CBytes(None, 0)
        buf = ctypes.create_string_buffer(x, max(1, len(x)))
        self._keep.append(buf)
        return _abi.CBytes(ctypes.addressof(buf), len(x))


def size(rpc: RPC) -> int:
    """RPC.Size()."""
    t = _Tables(rpc)
    return int(_abi.load().gsim_wire_size(ctypes.byref(t.rpc)))


def marshal(rpc: RPC) -> bytes:
    """RPC.Marshal()."""
    t = _Tables(rpc)
    lib = _abi.load()
    n = int(lib.gsim_wire_size(ctypes.byref(t.rpc)))
    out = ctypes.create_string_buffer(max(1, n))
    ln = ctypes.c_uint64()
    rc = lib.gsim_wire_encode(ctypes.byref(t.rpc), out, n, ctypes.byref(ln))
    if rc != 0:
        raise WireError(rc, "encode")
    return out.raw[:ln.value]


def fragment_rpc(rpc: RPC, limit: int) -> List[bytes]:
    """fragmentRPC(rpc, limit): the fragments, encoded.  Raises WireError
    (GSIM_EINVAL) when a message alone exceeds the limit."""
    t = _Tables(rpc)
    lib = _abi.load()
    ln, nf = ctypes.c_uint64(), ctypes.c_int32()
    rc = lib.gsim_wire_fragment(ctypes.byref(t.rpc), limit, None, 0, ctypes.byref(ln), None, 0, ctypes.byref(nf))
    if rc == _abi.GSIM_EINVAL:
        raise WireError(rc, f"a message exceeds limit {limit}")
    out = ctypes.create_string_buffer(max(1, ln.value))
    off = (ctypes.c_uint64 * (nf.value + 1))()
    rc = lib.gsim_wire_fragment(ctypes.byref(t.rpc), limit, out, ln.value, ctypes.byref(ln), off, nf.value,
                                ctypes.byref(nf))
    if rc != 0:
        raise WireError(rc, "fragment")
    raw = out.raw
    return [raw[off[k]:off[k + 1]] for k in range(nf.value)]


def _bytes_at(b: _abi.CBytes) -> Optional[bytes]:
    return None if not b.p else ctypes.string_at(b.p, b.n)


def unmarshal(data: bytes) -> RPC:
    """RPC.Unmarshal (gsim_wire_decode): the RPC encoded in `data`.  Raises
    WireError (GSIM_EINVAL) for a malformed RPC ("bogus rpc", comm.go:82)."""
    lib = _abi.load()
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    t = _abi.CWireTables()
    r = _abi.CWireRpc()
    rc = lib.gsim_wire_decode(buf, len(data), ctypes.byref(t), ctypes.byref(r))
    if rc == _abi.GSIM_ERANGE:                       # the counts needed: size the tables
        keep = []

        def arr(ct, n, name):
            a = (ct * max(1, n))()
            keep.append(a)
            setattr(t, name, ctypes.addressof(a))
            setattr(t, name + "_cap", n)
            return a
        subs = arr(_abi.CWireSub, r.nsubs, "subs")
        msgs = arr(_abi.CWireMsg, r.nmsgs, "msgs")
        ihave = arr(_abi.CWireIHave, r.nihave, "ihave")
        iwant = arr(_abi.CWireIWant, r.niwant, "iwant")
        graft = arr(_abi.CWireGraft, r.ngraft, "graft")
        prune = arr(_abi.CWirePrune, r.nprune, "prune")
        ids = arr(_abi.CBytes, r.nids, "ids")
        pxs = arr(_abi.CWirePx, r.npx, "px")
        rc = lib.gsim_wire_decode(buf, len(data), ctypes.byref(t), ctypes.byref(r))
    else:
        subs = msgs = ihave = iwant = graft = prune = ids = pxs = []
    if rc != 0:
        raise WireError(rc, "bogus rpc")
    out = RPC()
    for k in range(r.nsubs):
        out.subscriptions.append(SubOpts(None if subs[k].subscribe < 0 else bool(subs[k].subscribe),
                                         _bytes_at(subs[k].topic)))
    for k in range(r.nmsgs):
        m = msgs[k]
        out.publish.append(Message(*(_bytes_at(getattr(m, f)) for f in ("from_", "data", "seqno", "topic",
                                                                          "signature", "key"))))
    if r.has_control:
        c = ControlMessage()
        for k in range(r.nihave):
            g = ihave[k]
            c.ihave.append(ControlIHave(_bytes_at(g.topic), [_bytes_at(ids[g.id0 + q]) for q in range(g.nid)]))
        for k in range(r.niwant):
            g = iwant[k]
            c.iwant.append(ControlIWant([_bytes_at(ids[g.id0 + q]) for q in range(g.nid)]))
        for k in range(r.ngraft):
            c.graft.append(ControlGraft(_bytes_at(graft[k].topic)))
        for k in range(r.nprune):
            p = prune[k]
            c.prune.append(ControlPrune(_bytes_at(p.topic),
                                        [PeerInfo(_bytes_at(pxs[p.px0 + q].peer), _bytes_at(pxs[p.px0 + q].record))
                                         for q in range(p.npx)],
                                        p.backoff if p.has_backoff else None))
        out.control = c
    return out


def delimited(rpcs) -> bytes:
    """The varint-delimited stream of encoded RPCs (the sender's msgio varint
    writer, comm.go)."""
    out = bytearray()
    for b in rpcs:
        n = len(b)
        while n >= 0x80:
            out.append((n & 0x7F) | 0x80)
            n >>= 7
        out.append(n)
        out += b
    return bytes(out)


def frames(stream: bytes, max_size: int = 1 << 20):
    """gsim_wire_frames: the whole frames of a varint-delimited stream
    (msgio.NewVarintReaderSize(s, maxMessageSize), comm.go:64) and the bytes
    they use; raises WireError (GSIM_ERANGE) for a frame over max_size."""
    lib = _abi.load()
    buf = ctypes.create_string_buffer(bytes(stream), max(1, len(stream)))
    cap = max(1, len(stream))
    off = (ctypes.c_uint64 * cap)()
    ln = (ctypes.c_uint64 * cap)()
    n, used = ctypes.c_int32(), ctypes.c_uint64()
    rc = lib.gsim_wire_frames(buf, len(stream), max_size, off, ln, cap, ctypes.byref(n), ctypes.byref(used))
    if rc != 0:
        raise WireError(rc, "message too large" if rc == _abi.GSIM_ERANGE else "bad length prefix")
    return [bytes(stream[off[k]:off[k] + ln[k]]) for k in range(n.value)], used.value


def heartbeat_rpcs(engine, tick: int, p0: int, p1: int, topic_names, peer_ids: Optional[np.ndarray] = None,
                   prune_backoff_s: Optional[int] = None):
    """The RPCs senders [p0, p1) sent at heartbeat `tick` (after
    engine.heartbeat(tick), before the tick's first round), encoded on the
    device: a list of (from, to, bytes) in sender order, each sender's in
    its row order.  peer_ids: optional [N, L] uint8 peer ids (message ids are
    then peer_id(origin) || seqno, else the 8-byte big-endian gsim id)."""
    import torch
    lib = _abi.load()
    names = [_b(x) for x in topic_names]
    tn = (_abi.CBytes * max(1, len(names)))()
    keep = []
    for k, x in enumerate(names):
        buf = ctypes.create_string_buffer(x, max(1, len(x)))
        keep.append(buf)
        tn[k] = _abi.CBytes(ctypes.addressof(buf), len(x))
    nm = _abi.CWireNames()
    nm.topic_names = ctypes.addressof(tn)
    if peer_ids is not None:
        pid = np.ascontiguousarray(peer_ids, dtype=np.uint8)
        keep.append(pid)
        nm.peer_ids = pid.ctypes.data
        nm.peer_id_len = pid.shape[1]
    gp = engine.gossip if hasattr(engine, "gossip") else None
    if prune_backoff_s is None:
        prune_backoff_s = int(gp.PruneBackoff // 10**9) if gp is not None else 60
    nm.prune_backoff_s = prune_backoff_s
    n, nb = ctypes.c_int64(), ctypes.c_uint64()
    rc = lib.gsim_wire_heartbeat(engine.h, tick, p0, p1, ctypes.byref(nm), None, 0, None, 0, ctypes.byref(n),
                                 ctypes.byref(nb))
    if rc not in (0, _abi.GSIM_ERANGE):
        raise WireError(rc, (lib.gsim_last_error(engine.h) or b"").decode())
    dev = f"cuda:{engine.device}" if hasattr(engine, "device") else "cuda"
    out = torch.empty(max(1, nb.value), dtype=torch.uint8, device=dev)
    refs = torch.empty(max(1, n.value) * 24, dtype=torch.uint8, device=dev)
    rc = lib.gsim_wire_heartbeat(engine.h, tick, p0, p1, ctypes.byref(nm), out.data_ptr(), nb.value,
                                 refs.data_ptr(), n.value, ctypes.byref(n), ctypes.byref(nb))
    if rc != 0:
        raise WireError(rc, (lib.gsim_last_error(engine.h) or b"").decode())
    raw = out.cpu().numpy().tobytes()
    rv = np.frombuffer(refs.cpu().numpy().tobytes()[:n.value * 24], dtype=_abi.WIRE_REF_DTYPE)
    return [(int(r["from"]), int(r["to"]), raw[int(r["offset"]):int(r["offset"]) + int(r["len"])]) for r in rv]


def trace_batch(records: np.ndarray, topic_names, peer_ids: Optional[np.ndarray] = None,
                proto: bytes = b"/meshsub/1.1.0") -> bytes:
    """TraceEventBatch bytes (pb/trace.proto) of engine trace records
    (Engine.trace_read; gsim_trace_encode)."""
    lib = _abi.load()
    recs = np.ascontiguousarray(records)
    names = [_b(x) for x in topic_names]
    tn = (_abi.CBytes * max(1, len(names)))()
    keep = []
    for k, x in enumerate(names):
        buf = ctypes.create_string_buffer(x, max(1, len(x)))
        keep.append(buf)
        tn[k] = _abi.CBytes(ctypes.addressof(buf), len(x))
    nm = _abi.CWireNames()
    nm.topic_names = ctypes.addressof(tn)
    if peer_ids is not None:
        pid = np.ascontiguousarray(peer_ids, dtype=np.uint8)
        keep.append(pid)
        nm.peer_ids = pid.ctypes.data
        nm.peer_id_len = pid.shape[1]
    n = ctypes.c_uint64()
    ptr = recs.ctypes.data_as(ctypes.c_void_p) if len(recs) else None
    rc = lib.gsim_trace_encode(ptr, len(recs), ctypes.byref(nm), proto, None, 0, ctypes.byref(n))
    if rc not in (0, _abi.GSIM_ERANGE):
        raise WireError(rc, "gsim_trace_encode")
    out = ctypes.create_string_buffer(max(1, n.value))
    rc = lib.gsim_trace_encode(ptr, len(recs), ctypes.byref(nm), proto, out, n.value, ctypes.byref(n))
    if rc != 0:
        raise WireError(rc, "gsim_trace_encode")
    return out.raw[:n.value]


def trace_rpc_batch(rpcs, topic_names=(), peer_ids: Optional[np.ndarray] = None, timestamp: int = 0,
                    which: int = 3) -> bytes:
    """TraceEventBatch of the SendRPC (which bit 0) / RecvRPC (bit 1) /
    DropRPC (bit 2) events of encoded RPCs [(from, to, bytes)], e.g.
    heartbeat_rpcs' output (gsim_trace_rpc_encode)."""
    lib = _abi.load()
    raw = b"".join(r[2] for r in rpcs)
    refs = np.zeros(len(rpcs), dtype=_abi.WIRE_REF_DTYPE)
    off = 0
    for k, (frm, to, b) in enumerate(rpcs):
        refs[k]["from"], refs[k]["to"], refs[k]["len"], refs[k]["offset"] = frm, to, len(b), off
        off += len(b)
    names = [_b(x) for x in topic_names]
    tn = (_abi.CBytes * max(1, len(names)))()
    keep = []
    for k, x in enumerate(names):
        buf = ctypes.create_string_buffer(x, max(1, len(x)))
        keep.append(buf)
        tn[k] = _abi.CBytes(ctypes.addressof(buf), len(x))
    nm = _abi.CWireNames()
    nm.topic_names = ctypes.addressof(tn)
    if peer_ids is not None:
        pid = np.ascontiguousarray(peer_ids, dtype=np.uint8)
        keep.append(pid)
        nm.peer_ids = pid.ctypes.data
        nm.peer_id_len = pid.shape[1]
    rb = ctypes.create_string_buffer(raw, max(1, len(raw)))
    n = ctypes.c_uint64()
    rp = refs.ctypes.data if len(refs) else None
    rc = lib.gsim_trace_rpc_encode(rb, rp, len(refs), ctypes.byref(nm), timestamp, which, None, 0, ctypes.byref(n))
    if rc not in (0, _abi.GSIM_ERANGE):
        raise WireError(rc, "gsim_trace_rpc_encode")
    out = ctypes.create_string_buffer(max(1, n.value))
    rc = lib.gsim_trace_rpc_encode(rb, rp, len(refs), ctypes.byref(nm), timestamp, which, out, n.value,
                                   ctypes.byref(n))
    if rc != 0:
        raise WireError(rc, "gsim_trace_rpc_encode")
    return out.raw[:n.value]


def pb_tracer_stream(batch: bytes) -> bytes:
    """PBTracer's trace file (tracer.go:130-179) of a TraceEventBatch
    (trace_batch / trace_rpc_batch output): each TraceEvent varint-delimited
    (gsim_trace_delimited)."""
    lib = _abi.load()
    src = ctypes.create_string_buffer(bytes(batch), max(1, len(batch)))
    n = ctypes.c_uint64()
    rc = lib.gsim_trace_delimited(src, len(batch), None, 0, ctypes.byref(n))
    if rc not in (0, _abi.GSIM_ERANGE):
        raise WireError(rc, "not a TraceEventBatch")
    out = ctypes.create_string_buffer(max(1, n.value))
    rc = lib.gsim_trace_delimited(src, len(batch), out, n.value, ctypes.byref(n))
    if rc != 0:
        raise WireError(rc, "gsim_trace_delimited")
    return out.raw[:n.value]

