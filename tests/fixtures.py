"""Shared parameter fixtures and seeded random engine states (test infrastructure)."""
from __future__ import annotations

import numpy as np

from gsim import _abi
from gsim.params import Second
from gsim.presets import beacon_params, beacon_thresholds, beacon_topic  # noqa: F401  (re-exported)


def sybil_ips(n: int, frac: float, per_ip: int, rng) -> tuple:
    """Honest peers get a unique IP; a `frac` share of peers share one IP per `per_ip`."""
    ip_of = np.arange(n, dtype=np.uint32)
    syb = rng.permutation(n)[: int(n * frac)]
    ip_of[syb] = n + (np.arange(len(syb)) // per_ip)
    ips, inv = np.unique(ip_of, return_inverse=True)
    ip_ptr = np.arange(n + 1, dtype=np.uint32)
    return ip_ptr, inv.astype(np.uint32), len(ips)


def randomize_state(st, rng, now: int, retained_frac: float = 0.05):
    """Fill a NetState with adversarially varied counters, flags and times."""
    T, E = st.first.shape

    def counters(scale):
        x = rng.exponential(scale, size=(T, E))
        x[rng.random((T, E)) < 0.3] = 0.0
        x[rng.random((T, E)) < 0.05] = 0.0101    # just above DecayToZero: snaps to 0 after decay
        return x

    st.first[...] = counters(20.0)
    st.meshd[...] = counters(60.0)
    st.fail[...] = counters(50.0)
    st.invalid[...] = counters(2.0)
    st.tflags[...] = (rng.random((T, E)) < 0.3).astype(np.uint8) * _abi.TF_IN_MESH
    st.tflags[...] |= (rng.random((T, E)) < 0.5).astype(np.uint8) * _abi.TF_ACTIVE
    st.graft_time[...] = now - rng.integers(0, 4000 * Second, size=(T, E))
    st.mesh_time[...] = rng.integers(0, 4000 * Second, size=(T, E))
    st.bp[...] = np.where(rng.random(E) < 0.5, rng.exponential(8.0, E), 0.0)
    r = rng.random(E)
    st.estate[...] = _abi.ES_TRACKED | _abi.ES_CONNECTED
    st.estate[r < retained_frac] = _abi.ES_TRACKED
    st.estate[(r >= retained_frac) & (r < retained_frac * 1.2)] = 0
    st.expire[...] = now + rng.integers(-5 * Second, 5 * Second, size=E)
    st.expire[st.estate != _abi.ES_TRACKED] = 0
    untracked = st.estate == 0
    for f in ("first", "meshd", "fail", "invalid", "graft_time", "mesh_time", "tflags"):
        getattr(st, f)[:, untracked] = 0
    st.bp[untracked] = 0


def synthetic_state(st, rng, now: int, p_mesh: float):
    """Host twin of gsim_fill_synthetic's distributions (engine.hip
    k_fill_synthetic): a mostly healthy steady-state network — mesh links with
    probability p_mesh, graft times within the last hour, first deliveries
    U{0..1999}/4, mesh deliveries U{0..1599}/4 on mesh links, occasional
    failure penalties, rare invalid deliveries and behaviour penalties."""
    T, E = st.first.shape
    in_mesh = rng.random((T, E)) < p_mesh
    st.tflags[...] = np.where(in_mesh, _abi.TF_IN_MESH | _abi.TF_MESH, 0).astype(np.uint8)
    st.tflags[in_mesh & (rng.integers(0, 16, (T, E)) != 0)] |= _abi.TF_ACTIVE
    st.graft_time[...] = np.where(in_mesh, now - rng.integers(0, 3600, (T, E)) * Second, 0)
    st.mesh_time[...] = np.where(in_mesh, now - st.graft_time, 0)
    st.first[...] = rng.integers(0, 2000, (T, E)) * 0.25
    st.meshd[...] = np.where(in_mesh, rng.integers(0, 1600, (T, E)) * 0.25, 0.0)
    st.fail[...] = np.where(rng.integers(0, 8, (T, E)) == 0, rng.integers(0, 4000, (T, E)) * 0.125, 0.0)
    st.invalid[...] = np.where(rng.integers(0, 512, (T, E)) == 0, rng.integers(0, 64, (T, E)) * 0.125, 0.0)
    st.bp[...] = np.where(rng.integers(0, 16, E) == 0, rng.integers(0, 100, E) * 0.125, 0.0)
    st.estate[...] = _abi.ES_TRACKED | _abi.ES_CONNECTED
    st.expire[...] = 0
    st.backoff[...] = 0
