"""Host side of the query kernels: views passed across the C ABI, the autograd
Function behind ``NeuralPoints.query_feature`` and the fused SDF(+gradient) call
used by the tracker and mesher paths."""
import ctypes
from ctypes import c_void_p
import os

import numpy as np
import torch

from . import _lib

# partition queries into spatial tiles before the grid SDF query (PIN_QUERY_TILES=0 disables)
_TILE_QUERIES = os.environ.get("PIN_QUERY_TILES", "1") != "0"
_TILE_MIN = 65536  # below this the partition's two launches cost more than the locality returns


class _View:
    """A ctypes struct plus the tensors it points into (kept alive with it)."""

    def __init__(self, struct, keep):
        self.struct = struct
        self.keep = keep

    def ref(self):
        return ctypes.byref(self.struct)


def _f32(t):
    return None if t is None else t.detach().to(torch.float32).contiguous()


def hash_view(nm) -> _View:
    table = nm.buffer_pt_index
    cells = nm._cell_table()
    s = _lib.PinHash(table=table.data_ptr(), buffer_size=nm.buffer_size,
                     resolution=float(np.float32(nm.resolution)), num_cells=int(nm.neighbor_K),
                     cells=cells.data_ptr(), max_valid_dist2=float(np.float32(nm.max_valid_dist2)), reserved=0)
    return _View(s, (table, cells))


def points_view(records, features, positions, orientations, certainties, after_pgo, positions4=None) -> _View:
    """positions4: the positions as [rows, 4] f32 (optional; the training forward's neighbour
    position loads)."""
    features = _f32(features)
    positions = _f32(positions)
    orientations = _f32(orientations) if after_pgo else None
    certainties = _f32(certainties)
    if certainties is not None and certainties.numel() == 0:   # empty map: never read, must be non-NULL
        certainties = torch.zeros(1, dtype=torch.float32, device=certainties.device)
    s = _lib.PinPoints(records=records.data_ptr(), num_points=records.shape[0], features=features.data_ptr(),
                       positions=positions.data_ptr() if positions is not None else None,
                       orientations=orientations.data_ptr() if orientations is not None else None,
                       certainties=certainties.data_ptr() if certainties is not None else None,
                       rows=features.shape[0], after_pgo=int(bool(after_pgo)), reserved=0,
                       positions4=positions4.data_ptr() if positions4 is not None else None)
    v = _View(s, (records, features, positions, orientations, certainties, positions4))
    v.features = features
    return v


def tensor_key(ts):
    """Identity, storage pointer and version of each tensor (None kept): a derived view built from
    them is reusable while this tuple compares equal (in-place writes bump _version; the kernels'
    raw-pointer writes bump it through NeuralPoints.mark_modified)."""
    return tuple((id(t), t.data_ptr(), t._version) if t is not None else None for t in ts)


# decode on the f16 matrix cores (pin_mlp_pack image in PinMlp.packed; PIN_MLP_PACK=0: f32 VALU decoder)
_MLP_PACK = os.environ.get("PIN_MLP_PACK", "1") != "0"


def mlp_view(decoder, packed=False) -> _View:
    """PinMlp over a hidden_level=1, out_dim=1 geo decoder (model/decoder.py:16-57); cached on the
    decoder until a parameter is replaced or modified.  packed: also carry the pin_mlp_pack
    operand image (built once per decoder version) for the grid SDF kernels."""
    try:
        ps = (decoder.layers[0].weight, decoder.layers[0].bias, decoder.lout.weight, decoder.lout.bias)
    except (AttributeError, IndexError):
        ps = None
    if ps is not None and len(decoder.layers) == 1:
        key = (tensor_key(ps), float(decoder.sdf_scale))
        hit = decoder.__dict__.get("_pin_mlp_view")
        if hit is not None and hit[0] == key:
            v = hit[1]
        else:
            v = _mlp_view(decoder)
            decoder.__dict__["_pin_mlp_view"] = (key, v)
    else:
        v = _mlp_view(decoder)
    if packed and _MLP_PACK and not v.struct.packed:
        # one operand image per decoder, rewritten in stream order when the parameters change (a
        # training decoder's view is rebuilt every iteration; an older view reads the same
        # parameters in place, so it stays consistent with the image)
        buf = decoder.__dict__.get("_pin_mlp_pack_buf") if ps is not None else None
        if buf is None or buf.device != v.keep[0].device:
            # zeroed once: the image has padding bytes the pack never writes (images compare bytewise)
            buf = torch.zeros(_lib.MLP_PACK_BYTES, dtype=torch.uint8, device=v.keep[0].device)
            if ps is not None:
                decoder.__dict__["_pin_mlp_pack_buf"] = buf
        _lib.call("pin_mlp_pack", v.ref(), _lib.ptr(buf), _lib.stream(buf.device))
        v.struct.packed = buf.data_ptr()
        v.keep = v.keep + (buf,)
    return v


def mlp_view_repacked(decoder, packed_ptr) -> bool:
    """After a launch that stepped the decoder AND rewrote its operand image (the mapping loop's
    pin_adam_step_train re-packs it, bitwise pin_mlp_pack's image): cache the view under the
    parameters' new versions with that image attached, so the next mlp_view(packed=True) -- the
    tracker's -- does not pack again.  False (nothing cached) unless packed_ptr is this decoder's
    image buffer."""
    buf = decoder.__dict__.get("_pin_mlp_pack_buf")
    try:
        ps = (decoder.layers[0].weight, decoder.layers[0].bias, decoder.lout.weight, decoder.lout.bias)
    except (AttributeError, IndexError):
        return False
    if not _MLP_PACK or buf is None or buf.data_ptr() != packed_ptr or len(decoder.layers) != 1:
        return False
    v = _mlp_view(decoder)
    v.struct.packed = buf.data_ptr()
    v.keep = v.keep + (buf,)
    decoder.__dict__["_pin_mlp_view"] = ((tensor_key(ps), float(decoder.sdf_scale)), v)
    return True


def _mlp_view(decoder) -> _View:
    if len(decoder.layers) != 1 or decoder.out_dim != 1 or decoder.layers[0].bias is None:
        raise NotImplementedError("fused SDF kernels implement geo_mlp_level=1, out_dim=1, bias on")
    W1 = _f32(decoder.layers[0].weight)
    if tuple(W1.shape) != (_lib.HIDDEN_DIM, _lib.FEATURE_DIM + 3):
        raise NotImplementedError("fused SDF kernels implement an 11 -> 64 -> 1 decoder")
    b1 = _f32(decoder.layers[0].bias)
    W2 = _f32(decoder.lout.weight)
    b2 = _f32(decoder.lout.bias)
    s = _lib.PinMlp(W1=W1.data_ptr(), b1=b1.data_ptr(), W2=W2.data_ptr(), b2=b2.data_ptr(),
                    sdf_scale=float(np.float32(decoder.sdf_scale)), reserved=0)
    return _View(s, (W1, b1, W2, b2))


def _quat_rotate_passive(quat, v):
    """utils/tools.py:316-323 apply_quaternion_rotation (passive): v + w t + u x t, t = 2 u x v,
    u = -quat[1:]."""
    w = quat[..., 0:1]
    u = -quat[..., 1:]
    t = 2 * torch.linalg.cross(u, v)
    return v + w * t + torch.linalg.cross(u, t)


def _query_feature_restated(q, feats, ids, gids, records, positions, orientations, after_pgo, wf):
    """model/neural_points.py:577-662 over the neighbour sets the kernel found (ids: feature rows,
    gids: the candidates' records, -1 invalid), as differentiable torch ops in q and feats: the
    distance and IDW weights from the record (global) position, the decoder input's neighbour
    vector from the local position (flagged records, the global2local quirk) rotated after PGO.
    Used only to differentiate the backward itself (create_graph=True)."""
    qf = q.to(torch.float32)
    valid = gids >= 0
    g = gids.clamp(min=0).long()
    il = ids.clamp(min=0).long()
    rec = records.index_select(0, g.reshape(-1)).reshape(g.shape + (4,))
    bits = records.view(torch.int32)[:, 3].index_select(0, g.reshape(-1)).reshape(g.shape)
    pg = qf[:, None, :] - rec[..., :3]
    d2 = (pg[..., 0] * pg[..., 0] + pg[..., 1] * pg[..., 1]) + pg[..., 2] * pg[..., 2]
    u = torch.where(valid, 1.0 / (d2 + 1e-15), torch.zeros_like(d2))
    S = u.sum(1, keepdim=True)
    w = torch.where(valid, u / torch.where(S > 0, S, torch.ones_like(S)), torch.zeros_like(u))
    unf = valid & ((bits & _lib.RECORD_UNFAITHFUL) != 0)
    ploc = rec[..., :3]
    if bool(unf.any()):
        ploc = torch.where(unf[..., None], positions.index_select(0, il.reshape(-1)).reshape(il.shape + (3,)), ploc)
    v = qf[:, None, :] - ploc
    if after_pgo:
        v = _quat_rotate_passive(orientations.index_select(0, il.reshape(-1)).reshape(il.shape + (4,)), v)
    zero = torch.zeros((), dtype=torch.float32, device=q.device)
    v = torch.where(valid[..., None], v, zero)
    f = torch.where(valid[..., None], feats.index_select(0, il.reshape(-1)).reshape(il.shape + (feats.shape[1],)), zero)
    x = torch.cat((f, v), -1)
    out = (x * w[..., None]).sum(1) if wf else x
    return out, w


# second order through the autograd of _query_feature_restated instead of the native double
# backward (tests compare the two)
_QF_RESTATED = os.environ.get("PIN_QF_RESTATED", "0") == "1"


class _Saved:
    """The first backward's inputs kept by QueryFeatureFn (plain holder)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class QueryFeatureBwdFn(torch.autograd.Function):
    """The first-order backward of QueryFeatureFn as a differentiable op (create_graph=True):
    forward = pin_query_feature_bwd (grad_q and the grad_features scatter), backward =
    pin_query_feature_bwd2, the double backward in closed form (no ATen gathers)."""

    @staticmethod
    def forward(ctx, q, feats, g_feat, g_w, sv):
        n = sv.qd.shape[0]
        grad_q = torch.empty_like(sv.qd) if sv.need_q else torch.zeros((0, 3), dtype=torch.float32, device=q.device)
        grad_f = torch.zeros_like(sv.pv.features) if sv.need_f else torch.zeros((0, 8), dtype=torch.float32,
                                                                                  device=q.device)
        gf = g_feat.contiguous() if g_feat is not None else None
        gw = g_w.contiguous() if g_w is not None else None
        _lib.call("pin_query_feature_bwd", sv.pv.ref(), _lib.ptr(sv.qd), n, sv.nn_k, int(sv.wf), _lib.ptr(sv.ids),
                  _lib.ptr(sv.gids), _lib.ptr(sv.weights), _lib.ptr(gf), _lib.ptr(gw),
                  _lib.ptr(grad_q) if sv.need_q else None, _lib.ptr(grad_f) if sv.need_f else None, _lib.stream())
        ctx.save_for_backward(gf, gw)
        ctx.sv = sv
        ctx.has = (g_feat is not None, g_w is not None)
        if sv.need_q and sv.q_dtype != torch.float32:
            grad_q = grad_q.to(sv.q_dtype)
        return grad_q, grad_f

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, h_q, h_f):
        gf, gw = ctx.saved_tensors
        sv = ctx.sv
        n = sv.qd.shape[0]
        need_q, need_f, need_g, need_w = (ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                          ctx.needs_input_grad[2] and ctx.has[0], ctx.needs_input_grad[3] and ctx.has[1])
        up_q = h_q.to(torch.float32).contiguous() if (h_q is not None and sv.need_q) else None
        up_f = h_f.to(torch.float32).contiguous() if (h_f is not None and sv.need_f) else None
        dq = torch.empty_like(sv.qd) if need_q else None
        dg = torch.empty_like(gf) if need_g else None
        dw = torch.empty_like(gw) if need_w else None
        dF = torch.zeros_like(sv.pv.features) if need_f else None
        if up_q is None and up_f is None:
            return (torch.zeros_like(sv.q) if need_q else None, dF, torch.zeros_like(gf) if need_g else None,
                    torch.zeros_like(gw) if need_w else None, None)
        _lib.call("pin_query_feature_bwd2", sv.pv.ref(), _lib.ptr(sv.qd), n, sv.nn_k, int(sv.wf), _lib.ptr(sv.ids),
                  _lib.ptr(sv.gids), _lib.ptr(sv.weights), _lib.ptr(gf), _lib.ptr(gw), _lib.ptr(up_q), _lib.ptr(up_f),
                  _lib.ptr(dq), _lib.ptr(dg), _lib.ptr(dw), _lib.ptr(dF), _lib.stream())
        if dq is not None and sv.q_dtype != torch.float32:
            dq = dq.to(sv.q_dtype)
        return dq, dF, dg, dw, None


class QueryFeatureFn(torch.autograd.Function):
    """neural_points.py:528-674 forward on the GPU; backward = dL/dq and a float-atomic
    scatter of dL/dfeatures (the reference's autograd through index_put / gather).

    Second order (a caller differentiating the gradient, e.g. get_gradient with create_graph=True,
    utils/tools.py:174-184): the backward is then itself a differentiable op, QueryFeatureBwdFn,
    whose own backward is the closed-form double backward pin_query_feature_bwd2 (the fused
    mapping() evaluates the eikonal case in closed form too, PIN_TRAIN_EIK).  PIN_QF_RESTATED=1
    takes it by autograd over _query_feature_restated on the kernel's neighbour sets instead."""

    @staticmethod
    def forward(ctx, q, feats, hv, pv, nn_k, weighted_first, gv=None):
        qd = q.detach().to(torch.float32).contiguous()
        n = qd.shape[0]
        dev = qd.device
        D = _lib.FEATURE_DIM + 3
        feat = torch.empty((n, D) if weighted_first else (n, nn_k, D), dtype=torch.float32, device=dev)
        weights = torch.empty((n, nn_k), dtype=torch.float32, device=dev)
        nn_counts = torch.empty((n,), dtype=torch.int64, device=dev)
        cert = torch.empty((n,), dtype=torch.float32, device=dev)
        ids = torch.empty((n, nn_k), dtype=torch.int32, device=dev)
        gids = torch.empty((n, nn_k), dtype=torch.int32, device=dev)
        if gv is not None:
            _lib.call("pin_query_feature_fwd_grid", gv.ref(), pv.ref(), _lib.ptr(qd), n, nn_k, int(weighted_first),
                      _lib.ptr(feat), _lib.ptr(weights), _lib.ptr(nn_counts), _lib.ptr(cert), _lib.ptr(ids),
                      _lib.ptr(gids), _lib.stream())
        else:
            _lib.call("pin_query_feature_fwd", hv.ref(), pv.ref(), _lib.ptr(qd), n, nn_k, int(weighted_first),
                      _lib.ptr(feat), _lib.ptr(weights), _lib.ptr(nn_counts), _lib.ptr(cert), _lib.ptr(ids),
                      _lib.ptr(gids), _lib.stream())
        # q and feats themselves are kept for the differentiable (second-order) backward
        ctx.save_for_backward(q, feats, qd, ids, gids, weights)
        ctx.pv = pv
        ctx.nn_k = nn_k
        ctx.wf = weighted_first
        ctx.q_dtype = q.dtype
        ctx.mark_non_differentiable(nn_counts, cert, ids)
        return feat, weights, nn_counts, cert, ids

    @staticmethod
    def backward(ctx, g_feat, g_w, _g_nn, _g_cert, _g_ids):
        q, feats, qd, ids, gids, weights = ctx.saved_tensors
        need_q, need_f = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_q or need_f):
            return None, None, None, None, None, None, None
        if torch.is_grad_enabled() and not _QF_RESTATED:
            # create_graph=True: the backward as a differentiable op with a native double backward
            sv = _Saved(pv=ctx.pv, qd=qd, ids=ids, gids=gids, weights=weights, nn_k=ctx.nn_k, wf=ctx.wf,
                        need_q=need_q, need_f=need_f, q_dtype=ctx.q_dtype, q=q)
            gq, gf = QueryFeatureBwdFn.apply(q, feats, g_feat, g_w, sv)
            return (gq if need_q else None), (gf if need_f else None), None, None, None, None, None
        if torch.is_grad_enabled():   # create_graph=True: the backward must itself be differentiable
            pv = ctx.pv
            records, _, positions, orientations = pv.keep[0], pv.keep[1], pv.keep[2], pv.keep[3]
            with torch.enable_grad():
                out, w = _query_feature_restated(q, feats, ids, gids, records, positions, orientations,
                                                 bool(pv.struct.after_pgo), ctx.wf)
                outs, gos = [], []
                for o, go in ((out, g_feat), (w, g_w)):
                    if go is not None:
                        outs.append(o)
                        gos.append(go)
                inputs = [t for t, need in ((q, need_q), (feats, need_f)) if need]
                grads = list(torch.autograd.grad(outs, inputs, gos, create_graph=True, allow_unused=True))
            gq = grads.pop(0) if need_q else None
            gf = grads.pop(0) if need_f else None
            if need_q and gq is None:
                gq = torch.zeros_like(q)
            if need_f and gf is None:
                gf = torch.zeros_like(feats)
            return gq, gf, None, None, None, None, None
        n = qd.shape[0]
        grad_q = torch.empty_like(qd) if need_q else None
        grad_f = torch.zeros_like(ctx.pv.features) if need_f else None
        gf = g_feat.contiguous() if g_feat is not None else None
        gw = g_w.contiguous() if g_w is not None else None
        _lib.call("pin_query_feature_bwd", ctx.pv.ref(), _lib.ptr(qd), n, ctx.nn_k, int(ctx.wf), _lib.ptr(ids),
                  _lib.ptr(gids), _lib.ptr(weights), _lib.ptr(gf), _lib.ptr(gw), _lib.ptr(grad_q), _lib.ptr(grad_f),
                  _lib.stream())
        if grad_q is not None and ctx.q_dtype != torch.float32:
            grad_q = grad_q.to(ctx.q_dtype)
        return grad_q, grad_f, None, None, None, None, None


ORDER_STATE_BYTES = 65600   # PIN_ORDER_STATE_BYTES
_order_ws = {}


def order_workspace(n, device, stream_handle=None):
    """Workspace of pin_query_order / pin_query_sort: its state bytes must be zero before the
    first call and every call leaves them zero, so one zero-initialised buffer per (device,
    stream) is kept and grown (calls on one stream are ordered)."""
    key = (str(device), _lib.stream(device).value if stream_handle is None else stream_handle)
    need = ORDER_STATE_BYTES + 8 * max(n, 1)
    ws = _order_ws.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.zeros((max(need, 2 * (ws.numel() if ws is not None else 0)),), dtype=torch.uint8, device=device)
        _order_ws[key] = ws
    return ws


def query_order(gv, q):
    """pin_query_order: a tile-grouped processing order for the queries q [N,3] (device int32)."""
    n = q.shape[0]
    order = torch.empty((n,), dtype=torch.int32, device=q.device)
    ws = order_workspace(n, q.device)
    _lib.call("pin_query_order", gv.ref(), _lib.ptr(q), n, _lib.ptr(order), _lib.ptr(ws), _lib.stream())
    return order


_stable_ws = {}


def query_sort(gv, q, out=None, stable=False):
    """pin_query_sort: the queries q [N,3] in tile order as [N,4] f32 rows {x, y, z, bits(index)}.
    stable: pin_query_sort_stable (inside a tile the input order is kept: a deterministic order)."""
    n = q.shape[0]
    q4 = out if out is not None else torch.empty((n, 4), dtype=torch.float32, device=q.device)
    if stable:
        need = int(_lib.load().pin_query_sort_stable_workspace_bytes(max(n, 1)))
        if need < 0:
            raise RuntimeError("pin_query_sort_stable_workspace_bytes failed")
        key = str(q.device)
        ws = _stable_ws.get(key)
        if ws is None or ws.numel() < need:
            ws = _stable_ws[key] = torch.empty((need,), dtype=torch.uint8, device=q.device)
        _lib.call("pin_query_sort_stable", gv.ref(), _lib.ptr(q), n, _lib.ptr(q4), None, _lib.ptr(ws),
                  _lib.stream(q.device))
        return q4
    ws = order_workspace(n, q.device)
    _lib.call("pin_query_sort", gv.ref(), _lib.ptr(q), n, _lib.ptr(q4), None, _lib.ptr(ws), _lib.stream(q.device))
    return q4


def query_sdf(nm, decoder, points, query_locally=True, want_grad=True, zero_empty=False, want_std=False,
              want_certainty=True, nn_k=None, weighted_first=None, sorted_rows=None, out_order="input"):
    """Fused query_feature + Decoder.sdf (+ analytic dSDF/dq) in one kernel.

    Returns (sdf [N], grad [N,3] or None, nn_count [N] int32, certainty [N] or None,
    sdf_std [N] or None).  Semantics: utils/tracker.py:176-260 (query_locally=True) and
    utils/mesher.py:41-136 (query_locally=False, zero_empty=True).  sorted_rows: q already sorted
    by query_sort.  out_order "tile": where the batch is tile-sorted (grid backend, N >= _TILE_MIN)
    the outputs stay in tile order (coalesced stores) and a sixth value, the sorted rows q4 [N,4]
    {x, y, z, bits(index)}, says which query each output row belongs to; otherwise (and with
    "input") the outputs are in input order and the sixth value is None."""
    if out_order not in ("input", "tile"):
        raise ValueError("out_order must be 'input' or 'tile'")
    _lib.require_device(points)
    q = points.detach().to(torch.float32).contiguous()
    n = q.shape[0]
    dev = q.device
    nn_k = int(nm.config.query_nn_k if nn_k is None else nn_k)
    wf = bool(nm.config.weighted_first if weighted_first is None else weighted_first)
    mode = "local" if query_locally else "global"
    hv, pv = nm._views(mode, query_locally)
    mv = mlp_view(decoder, packed=want_grad)
    sdf = torch.empty(n, dtype=torch.float32, device=dev)
    grad = torch.empty((n, 3), dtype=torch.float32, device=dev) if want_grad else None
    nn_count = torch.empty(n, dtype=torch.int32, device=dev)
    cert = torch.empty(n, dtype=torch.float32, device=dev) if want_certainty else None
    std = torch.empty(n, dtype=torch.float32, device=dev) if (want_std and not wf) else None
    tile_out = False
    if nm.backend() == "grid":
        gv = nm.grid_view(mode, True)
        if sorted_rows is not None:
            _lib.call("pin_query_sdf_grid_sorted", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(sorted_rows), n, nn_k,
                      int(wf), int(zero_empty), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn_count), _lib.ptr(cert),
                      _lib.ptr(std), _lib.stream(dev))
        elif _TILE_QUERIES and n >= _TILE_MIN:
            # tile sort + sorted query in one call (pin_query_sdf_grid_tiled_ex)
            q4 = torch.empty((n, 4), dtype=torch.float32, device=dev)
            ws = order_workspace(n, dev)
            tile_out = out_order == "tile"
            _lib.call("pin_query_sdf_grid_tiled_ex", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, nn_k, int(wf),
                      int(zero_empty), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn_count), _lib.ptr(cert),
                      _lib.ptr(std), _lib.ptr(q4), _lib.ptr(ws), _lib.PIN_QUERY_OUT_TILE if tile_out else 0,
                      _lib.stream(dev))
        else:
            _lib.call("pin_query_sdf_grid", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, nn_k, int(wf),
                      int(zero_empty), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn_count), _lib.ptr(cert),
                      _lib.ptr(std), None, _lib.stream())
    else:
        _lib.call("pin_query_sdf", hv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, nn_k, int(wf), int(zero_empty),
                  _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn_count), _lib.ptr(cert), _lib.ptr(std), _lib.stream())
    if want_std and wf:
        std = torch.zeros(n, dtype=torch.float32, device=dev)
    if out_order == "tile":
        return sdf, grad, nn_count, cert, std, (q4 if tile_out else None)
    return sdf, grad, nn_count, cert, std
