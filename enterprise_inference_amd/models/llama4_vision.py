"""Llama-4 vision path: image tiles -> ViT encoder -> pixel-shuffle adapter -> projector into
the text model's embedding space (Llama-4-Scout-17B-16E-Instruct is multimodal; reference
core/lib/models/model-selection.sh:33).

Pipeline (checkpoint names ``vision_model.*`` / ``multi_modal_projector.*``):
  preprocess (here, PIL + numpy): best-fit tile canvas of up to ``max_tiles`` 336x336 tiles
    without distortion, pad, normalise (mean 0.5 / std 0.5), split into tiles, plus a global
    thumbnail tile when there is more than one;
  encoder (per tile): 14x14 patch unfold + linear, class token, learned positions, pre-norm,
    N x [LayerNorm -> MHA with 2-D rotary (x, y patch coordinates, complex pairs) -> LayerNorm
    -> GELU MLP], post-norm, drop the class token;
  adapter: pixel shuffle (ratio 0.5: 576 patches -> 144 tokens of 4x the width) -> GELU MLP;
  projector: linear to the text hidden size.
Each image becomes ``tiles x 144`` embeddings that replace the ``<|patch|>`` placeholder
tokens of its prompt expansion (``expand_image_prompt``), written over the token embeddings
of those positions in the prefill batch (models/llama.py forward, ``md.mm_rows``).

Linear layers run through ops.gemm (hipBLASLt / skinny HIP kernels), LayerNorm through the HIP
layer-norm kernel, attention as batched GEMMs (hipBLASLt) around an fp32 softmax (577
non-causal tokens per tile, once per image -- not a hot path).
"""

from __future__ import annotations

import base64
import contextlib
import io
import os
import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import gemm

TILE = 336
PATCH = 14


# ----------------------------------------------------------------------------- preprocessing
def _supported_canvases(max_tiles: int, tile: int = TILE) -> List[Tuple[int, int]]:
    out = []
    for n in range(max_tiles, 0, -1):
        for h in range(1, n + 1):
            if n % h == 0:
                out.append((h * tile, (n // h) * tile))
    return sorted(set(out))


def best_fit_canvas(h: int, w: int, max_tiles: int, tile: int = TILE) -> Tuple[int, int]:
    """Smallest upscale >= 1 (else the least downscale), ties -> smallest area."""
    cands = _supported_canvases(max_tiles, tile)
    scales = [min(ch / h, cw / w) for ch, cw in cands]
    ups = [s for s in scales if s >= 1]
    sel = min(ups) if ups else max(scales)
    best = [c for c, s in zip(cands, scales) if s == sel]
    return min(best, key=lambda c: c[0] * c[1])


MAX_IMAGE_BYTES = int(os.environ.get("EIA_MAX_IMAGE_BYTES", 20 << 20))
MAX_IMAGE_PIXELS = int(os.environ.get("EIA_MAX_IMAGE_PIXELS", 64 << 20))


def _remote_media_policy():
    """(enabled, allowed domains or None, private addresses allowed) from the environment:
    EIA_DISABLE_REMOTE_MEDIA=1 turns http(s) image URLs off, EIA_ALLOWED_MEDIA_DOMAINS
    (comma list) restricts the hosts (vLLM's --allowed-media-domains), and loopback /
    private / link-local targets are refused unless EIA_ALLOW_PRIVATE_MEDIA=1 (the server
    must not become a proxy into the cluster network)."""
    off = os.environ.get("EIA_DISABLE_REMOTE_MEDIA", "0") not in ("0", "", "false")
    doms = [d.strip().lower() for d in os.environ.get("EIA_ALLOWED_MEDIA_DOMAINS", "").split(",")
            if d.strip()]
    priv = os.environ.get("EIA_ALLOW_PRIVATE_MEDIA", "0") not in ("0", "", "false")
    return not off, (doms or None), priv


def _non_public(ip) -> bool:
    return (ip.is_private or ip.is_loopback or ip.is_link_local or ip.is_reserved or
            ip.is_multicast or ip.is_unspecified)


def _check_url(url: str):
    """Apply the media policy to ``url``.  Returns the one validated address the fetch must
    dial (``None`` when private targets are allowed and the name is resolved by the client
    as usual).  Resolving once and connecting to exactly that address closes the DNS
    rebinding window between the check and the connection."""
    import ipaddress
    import socket
    from urllib.parse import urlparse

    enabled, domains, allow_private = _remote_media_policy()
    if not enabled:
        raise ValueError("remote image URLs are disabled on this server")
    u = urlparse(url)
    if u.scheme not in ("http", "https"):
        raise ValueError("image URL must be http(s)")
    host = (u.hostname or "").lower()
    if not host:
        raise ValueError("image URL has no host")
    if domains is not None and not any(host == d or host.endswith("." + d) for d in domains):
        raise ValueError(f"image host {host!r} is not in the allowed media domains")
    if allow_private:
        return None
    addrs = [ipaddress.ip_address(info[4][0].split("%")[0])
             for info in socket.getaddrinfo(host, u.port or (443 if u.scheme == "https" else 80),
                                            type=socket.SOCK_STREAM)]
    if not addrs:
        raise ValueError(f"image host {host!r} does not resolve")
    for ip in addrs:
        if _non_public(ip):
            raise ValueError(f"image host {host!r} resolves to a non-public address")
    return addrs[0]


def _pinned_request(url: str, ip):
    """(url with the host replaced by the validated address, headers, extensions): the TCP
    connection goes to ``ip`` while Host, TLS SNI and certificate checks use the name."""
    from urllib.parse import urlparse, urlunparse

    u = urlparse(url)
    host = u.hostname
    lit = f"[{ip}]" if ip.version == 6 else str(ip)
    netloc = lit + (f":{u.port}" if u.port else "")
    hdr_host = (f"[{host}]" if ":" in host else host) + (f":{u.port}" if u.port else "")
    ext = {"sni_hostname": host} if u.scheme == "https" else {}
    return urlunparse(u._replace(netloc=netloc)), {"Host": hdr_host}, ext


def _proxy_for(url: str) -> Optional[str]:
    """The egress proxy the environment configures for ``url`` (HTTP(S)_PROXY / ALL_PROXY,
    honouring NO_PROXY against the host NAME), or None for a direct connection."""
    import urllib.request
    from urllib.parse import urlparse

    u = urlparse(url)
    proxies = urllib.request.getproxies()
    proxy = proxies.get(u.scheme) or proxies.get("all")
    if not proxy or urllib.request.proxy_bypass(u.hostname or ""):
        return None
    return proxy


@contextlib.contextmanager
def _open_stream(url: str, headers: dict, extensions: dict, timeout: float,
                 trust_env: bool = False):
    """One streamed GET (no redirect following) with per-request transport extensions.
    ``trust_env`` False (the pinned, direct form) ignores HTTP(S)_PROXY: the connection must go
    to the address the policy check validated, not to a proxy."""
    import httpx

    with httpx.Client(timeout=timeout, follow_redirects=False, trust_env=trust_env) as client:
        req = client.build_request("GET", url, headers=headers, extensions=extensions)
        r = client.send(req, stream=True)
        try:
            yield r
        finally:
            r.close()


class _ProxiedResponse:
    """The slice of an httpx streamed response ``fetch_image_bytes`` reads, over an
    http.client response."""

    def __init__(self, resp):
        self._r = resp
        self.status_code = resp.status
        self.headers = {k.lower(): v for k, v in resp.getheaders()}
        self.is_redirect = resp.status in (301, 302, 303, 307, 308) and "location" in self.headers
        self.extensions = {}

    def raise_for_status(self) -> None:
        if self.status_code >= 400:
            raise ValueError(f"image fetch failed: HTTP {self.status_code}")

    def iter_bytes(self, size: int = 1 << 16):
        while True:
            b = self._r.read(size)
            if not b:
                return
            yield b


@contextlib.contextmanager
def _open_proxied_stream(url: str, headers: dict, extensions: dict, timeout: float, proxy: str):
    """One GET of the PINNED target ``url`` (host = the validated address) through the egress
    proxy, so the proxy dials exactly the address the policy check vetted -- it never
    resolves the name itself, which would reopen the DNS-rebinding window:

    * http: absolute-form request ``GET http://<ip>:<port>/path`` with Host = the name;
    * https: ``CONNECT <ip>:<port>``, then TLS inside the tunnel with SNI and certificate
      verification against the NAME (``sni_hostname``).  httpx's tunnel takes the TLS server
      name from the CONNECT target, so this path is built on http.client.
    """
    import base64 as b64
    import http.client
    import ssl
    from urllib.parse import unquote, urlparse

    u, pu = urlparse(url), urlparse(proxy)
    if pu.scheme not in ("http", ""):
        raise ValueError(f"unsupported egress proxy scheme {pu.scheme!r}")
    auth = {}
    if pu.username:
        cred = f"{unquote(pu.username)}:{unquote(pu.password or '')}".encode()
        auth = {"Proxy-Authorization": "Basic " + b64.b64encode(cred).decode()}
    port = u.port or (443 if u.scheme == "https" else 80)
    path = (u.path or "/") + (f"?{u.query}" if u.query else "")
    if u.scheme == "https":
        name = extensions["sni_hostname"]
        ctx = ssl.create_default_context()

        class _Tunnel(http.client.HTTPSConnection):
            def connect(self):
                http.client.HTTPConnection.connect(self)       # TCP to the proxy + CONNECT
                self.sock = ctx.wrap_socket(self.sock, server_hostname=name)

        conn = _Tunnel(pu.hostname, pu.port or 3128, timeout=timeout, context=ctx)
        conn.set_tunnel(u.hostname, port, headers=auth)
        conn.request("GET", path, headers=headers)
    else:
        conn = http.client.HTTPConnection(pu.hostname, pu.port or 3128, timeout=timeout)
        conn.request("GET", url, headers={**headers, **auth})
    try:
        yield _ProxiedResponse(conn.getresponse())
    finally:
        conn.close()


def fetch_image_bytes(url: str, max_bytes: Optional[int] = None, timeout: float = 30.0) -> bytes:
    """Download an image URL with the media policy above and a byte cap (streamed: a huge or
    endless body is cut off at ``max_bytes`` instead of being buffered).  Redirects are
    followed by hand so every hop passes the same checks, and every hop connects to the
    address its check validated (no second DNS lookup an attacker's resolver could answer
    with an internal address)."""
    import ipaddress

    cap = MAX_IMAGE_BYTES if max_bytes is None else max_bytes
    for _ in range(5):
        ip = _check_url(url)
        # Behind an egress proxy (enterprise clusters, HTTP(S)_PROXY not bypassed by NO_PROXY
        # for the name) the PINNED target goes through the proxy: the proxy dials the address
        # validated above (CONNECT <ip> / absolute-form http://<ip>), TLS still verifies the
        # name.  The peer check cannot apply there (the peer is the proxy).  Direct fetches
        # dial the validated address with the environment's proxy settings ignored.
        proxy = _proxy_for(url) if ip is not None else None
        if ip is None:
            target, headers, ext = url, {}, {}
        else:
            target, headers, ext = _pinned_request(url, ip)
        opener = (_open_proxied_stream(target, headers, ext, timeout, proxy) if proxy
                  else _open_stream(target, headers, ext, timeout, trust_env=ip is None))
        with opener as r:
            if ip is not None and not proxy:   # defence in depth: peer is the checked address
                stream = r.extensions.get("network_stream")
                peer = stream.get_extra_info("server_addr") if stream is not None else None
                if peer and ipaddress.ip_address(str(peer[0]).split("%")[0]) != ip:
                    raise ValueError("image fetch connected to an unexpected address")
            if r.is_redirect:      # relative locations resolve against the NAME, not the IP
                from urllib.parse import urljoin
                url = urljoin(url, r.headers["location"])
                continue
            r.raise_for_status()
            n = int(r.headers.get("content-length") or 0)
            if n > cap:
                raise ValueError(f"image is {n} bytes (limit {cap})")
            buf = bytearray()
            for chunk in r.iter_bytes():
                buf += chunk
                if len(buf) > cap:
                    raise ValueError(f"image exceeds {cap} bytes")
            return bytes(buf)
    raise ValueError("too many redirects")


def load_image(src) -> "object":
    """PIL image from a PIL image, raw bytes, a data: URL, an http(s) URL or a local path.
    Decompression bombs are refused (``EIA_MAX_IMAGE_PIXELS``)."""
    from PIL import Image

    Image.MAX_IMAGE_PIXELS = MAX_IMAGE_PIXELS
    if hasattr(src, "convert"):
        return src.convert("RGB")
    if isinstance(src, (bytes, bytearray)):
        return Image.open(io.BytesIO(src)).convert("RGB")
    s = str(src)
    if s.startswith("data:"):
        data = base64.b64decode(s.split(",", 1)[1])
        if len(data) > MAX_IMAGE_BYTES:
            raise ValueError(f"image exceeds {MAX_IMAGE_BYTES} bytes")
        return Image.open(io.BytesIO(data)).convert("RGB")
    if s.startswith(("http://", "https://")):
        return Image.open(io.BytesIO(fetch_image_bytes(s))).convert("RGB")
    return Image.open(s).convert("RGB")


def preprocess(image, max_tiles: int = 16,
               tile: int = TILE) -> Tuple[torch.Tensor, Tuple[int, int]]:
    """-> (pixel_values [tiles, 3, tile, tile] fp32, (tiles_h, tiles_w))."""
    from PIL import Image

    TILE = tile                                                     # noqa: N806
    img = load_image(image)
    w, h = img.size
    ch, cw = best_fit_canvas(h, w, max_tiles, tile)
    s = min(ch / h, cw / w)
    nh, nw = min(ch, max(1, math.floor(h * s))), min(cw, max(1, math.floor(w * s)))
    canvas = np.zeros((ch, cw, 3), np.float32)
    canvas[:nh, :nw] = np.asarray(img.resize((nw, nh), Image.BILINEAR), np.float32)
    th, tw = ch // TILE, cw // TILE

    def norm(a):
        return (a / 255.0 - 0.5) / 0.5

    tiles = [norm(canvas[y * TILE:(y + 1) * TILE, x * TILE:(x + 1) * TILE])
             for y in range(th) for x in range(tw)]
    if th * tw > 1:
        tiles.append(norm(np.asarray(img.resize((TILE, TILE), Image.BILINEAR), np.float32)))
    pv = torch.from_numpy(np.stack(tiles)).permute(0, 3, 1, 2).contiguous()
    return pv, (th, tw)


def expand_image_prompt(aspect: Tuple[int, int], tokens_per_tile: int) -> str:
    """The placeholder text one image expands to (Llama-4 prompt format)."""
    th, tw = aspect
    s = "<|image_start|>"
    if th * tw > 1:
        for _ in range(th):
            for x in range(tw):
                s += "<|patch|>" * tokens_per_tile
                if x < tw - 1:
                    s += "<|tile_x_separator|>"
            s += "<|tile_y_separator|>"
    s += "<|image|>" + "<|patch|>" * tokens_per_tile + "<|image_end|>"
    return s


# ----------------------------------------------------------------------------- encoder
def _linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    shp = x.shape
    y = gemm.linear(x.reshape(-1, shp[-1]), w, b)
    return y.reshape(*shp[:-1], w.shape[0])


def _ln(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    from ..ops.norm import layer_norm
    shp = x.shape
    return layer_norm(x.reshape(-1, shp[-1]).contiguous(), w, b, eps).reshape(shp)


def pixel_shuffle(x: torch.Tensor, ratio: float) -> torch.Tensor:
    B, N, C = x.shape
    side = int(math.isqrt(N))
    x = x.view(B, side, side, C)
    x = x.view(B, side, int(side * ratio), int(C / ratio)).permute(0, 2, 1, 3).contiguous()
    x = x.view(B, int(side * ratio), int(side * ratio), int(C / ratio ** 2))
    return x.permute(0, 2, 1, 3).contiguous().view(B, -1, x.shape[-1])


class _P(nn.Module):
    """Parameter holder with HF-compatible names."""

    def __init__(self, **shapes):
        super().__init__()
        for k, (shape, dtype, device) in shapes.items():
            self.register_parameter(k, nn.Parameter(torch.empty(shape, dtype=dtype, device=device),
                                                    requires_grad=False))


class Llama4VisionTower(nn.Module):
    def __init__(self, vcfg: dict, text_hidden: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = vcfg
        D = vcfg["hidden_size"]
        I = vcfg["intermediate_size"]
        self.heads = vcfg["num_attention_heads"]
        self.hd = D // self.heads
        self.image_size = vcfg.get("image_size", TILE)
        self.patch = vcfg.get("patch_size", PATCH)
        self.side = self.image_size // self.patch
        self.ratio = vcfg.get("pixel_shuffle_ratio", 0.5)
        self.tokens_per_tile = int(self.side * self.side * self.ratio ** 2)
        pin = vcfg["projector_input_dim"]
        pout = vcfg["projector_output_dim"]
        ch = vcfg.get("num_channels", 3)
        kw = dict(dtype=dtype, device=device)
        t = lambda *s: (s, dtype, device)                               # noqa: E731
        self.patch_embedding = nn.Module()
        self.patch_embedding.linear = _P(weight=t(D, ch * self.patch * self.patch))
        self.class_embedding = nn.Parameter(torch.empty(D, **kw), requires_grad=False)
        self.positional_embedding_vlm = nn.Parameter(
            torch.empty(self.side * self.side + 1, D, **kw), requires_grad=False)
        self.layernorm_pre = _P(weight=t(D), bias=t(D))
        self.layernorm_post = _P(weight=t(D), bias=t(D))
        layers = nn.ModuleList()
        for _ in range(vcfg["num_hidden_layers"]):
            L = nn.Module()
            L.input_layernorm = _P(weight=t(D), bias=t(D))
            L.post_attention_layernorm = _P(weight=t(D), bias=t(D))
            L.self_attn = nn.Module()
            for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
                setattr(L.self_attn, n, _P(weight=t(D, D), bias=t(D)))
            L.mlp = nn.Module()
            L.mlp.fc1 = _P(weight=t(I, D), bias=t(I))
            L.mlp.fc2 = _P(weight=t(D, I), bias=t(D))
            layers.append(L)
        self.model = nn.Module()
        self.model.layers = layers
        self.vision_adapter = nn.Module()
        self.vision_adapter.mlp = nn.Module()
        self.vision_adapter.mlp.fc1 = _P(weight=t(pin, I))      # in: D / ratio^2 == I
        self.vision_adapter.mlp.fc2 = _P(weight=t(pout, pout))
        self.projector = _P(weight=t(text_hidden, vcfg["vision_output_dim"]))
        theta = vcfg.get("rope_theta") or (vcfg.get("rope_parameters") or {}).get("rope_theta",
                                                                                  10000.0)
        self.register_buffer("freqs", self._freqs(float(theta), device), persistent=False)

    def _freqs(self, theta: float, device) -> torch.Tensor:
        """cos/sin [patches + 1, hd/2] of the 2-D rotary (x then y frequencies, class = 0)."""
        idx = self.side
        img_idx = torch.arange(idx * idx).reshape(-1, 1)
        img_idx = torch.cat([img_idx, img_idx[:1]], 0)
        img_idx[-1, -1] = -2
        fx, fy = img_idx % idx, img_idx // idx
        fd = self.hd // 2
        rf = 1.0 / (theta ** (torch.arange(0, fd, 2)[: fd // 2].float() / fd))
        ax = ((fx + 1)[..., None] * rf[None, None, :]).repeat_interleave(2, dim=-1)
        ay = ((fy + 1)[..., None] * rf[None, None, :]).repeat_interleave(2, dim=-1)
        ang = torch.cat([ax, ay], -1).float()[..., ::2]
        ang = ang.masked_fill(img_idx.reshape(-1, 1, 1) < 0, 0).reshape(idx * idx + 1, -1)
        return torch.stack([torch.cos(ang), torch.sin(ang)], -1).to(device)   # [N, hd/2, 2]

    def _rope(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, N, H, hd]: interleaved pairs rotated by the per-patch angles."""
        cs = self.freqs.to(x.device)
        c, s = cs[..., 0][None, :, None, :], cs[..., 1][None, :, None, :]
        xf = x.float().reshape(*x.shape[:-1], -1, 2)
        a, b = xf[..., 0], xf[..., 1]
        out = torch.stack([a * c - b * s, a * s + b * c], -1).flatten(-2)
        return out.to(x.dtype)

    @torch.no_grad()
    def forward(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """pixel_values [tiles, 3, S, S] -> projected embeddings [tiles * tokens_per_tile, H]."""
        dt = self.class_embedding.dtype
        x = pixel_values.to(self.class_embedding.device, dt)
        T = x.shape[0]
        p = F.unfold(x, kernel_size=self.patch, stride=self.patch).transpose(1, 2)   # [T, N, C*p*p]
        h = _linear(p.contiguous(), self.patch_embedding.linear.weight)
        h = torch.cat([h, self.class_embedding.expand(T, 1, -1)], 1)
        h = h + self.positional_embedding_vlm
        h = _ln(h, self.layernorm_pre.weight, self.layernorm_pre.bias)
        N = h.shape[1]
        for L in self.model.layers:
            r = h
            y = _ln(h, L.input_layernorm.weight, L.input_layernorm.bias)
            a = L.self_attn
            q = self._rope(_linear(y, a.q_proj.weight, a.q_proj.bias).view(T, N, self.heads, self.hd))
            k = self._rope(_linear(y, a.k_proj.weight, a.k_proj.bias).view(T, N, self.heads, self.hd))
            v = _linear(y, a.v_proj.weight, a.v_proj.bias).view(T, N, self.heads, self.hd)
            # non-causal MHA as two batched library GEMMs around an fp32 softmax
            s = torch.matmul(q.transpose(1, 2), k.permute(0, 2, 3, 1)).float() * self.hd ** -0.5
            o = torch.matmul(torch.softmax(s, -1).to(v.dtype), v.transpose(1, 2))
            o = o.transpose(1, 2).reshape(T, N, -1)
            h = r + _linear(o, a.o_proj.weight, a.o_proj.bias)
            y = _ln(h, L.post_attention_layernorm.weight, L.post_attention_layernorm.bias)
            y = F.gelu(_linear(y, L.mlp.fc1.weight, L.mlp.fc1.bias))
            h = h + _linear(y, L.mlp.fc2.weight, L.mlp.fc2.bias)
        h = _ln(h, self.layernorm_post.weight, self.layernorm_post.bias)[:, :-1]
        h = pixel_shuffle(h, self.ratio)
        m = self.vision_adapter.mlp
        h = F.gelu(_linear(F.gelu(_linear(h, m.fc1.weight)), m.fc2.weight))
        out = _linear(h.reshape(-1, h.shape[-1]), self.projector.weight)
        return out

    def load_weight(self, name: str, tensor: torch.Tensor) -> bool:
        """HF names 'vision_model.<x>' / 'multi_modal_projector.linear_1.weight'."""
        if name.startswith("multi_modal_projector.linear_1."):
            tgt = self.projector.weight
        else:
            rest = name[len("vision_model."):]
            tgt = self
            try:
                for part in rest.split("."):
                    tgt = getattr(tgt, part) if not part.isdigit() else tgt[int(part)]
            except (AttributeError, IndexError):
                return False
        if not isinstance(tgt, torch.Tensor) or tgt.shape != tensor.shape:
            raise ValueError(f"vision weight {name}: shape {tuple(tensor.shape)} vs "
                             f"{tuple(getattr(tgt, 'shape', ()))}")
        tgt.data.copy_(tensor.to(tgt.dtype))
        return True


def image_positions(token_ids: Sequence[int], image_token_id: int) -> List[int]:
    return [i for i, t in enumerate(token_ids) if t == image_token_id]
