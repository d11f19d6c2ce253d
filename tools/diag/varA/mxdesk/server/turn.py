"""TURN/STUN RTC configuration (reference README.md:65-143, xgl.yml:85-109).

Three credential modes, as in the reference/selkies:
  * shared secret (coturn ``use-auth-secret``): time-limited username ``<expiry>:<user>``
    and password ``base64(HMAC-SHA1(secret, username))`` (README.md:85-113);
  * legacy long-term username/password (README.md:115-143);
  * TURN REST URI: credentials fetched from an HTTP service (selkies ``--turn_rest_uri``).
The result is the RTCConfiguration JSON served on ``/turn`` (``iceServers`` list).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time
from typing import Any


def hmac_credentials(secret: str, user: str = "mxdesk", ttl_s: int = 86400, now: float | None = None) -> tuple[str, str]:
    expiry = int((time.time() if now is None else now) + ttl_s)
    username = f"{expiry}:{user}"
    digest = hmac.new(secret.encode(), username.encode(), hashlib.sha1).digest()
    return username, base64.b64encode(digest).decode()


def turn_urls(host: str, port: int, protocol: str = "udp", tls: bool = False) -> list[str]:
    scheme = "turns" if tls else "turn"
    return [f"{scheme}:{host}:{port}?transport={protocol.lower()}"]


def rtc_config(cfg: Any, user: str = "mxdesk", now: float | None = None) -> dict:
    """Build the RTC configuration from a mxdesk Config (or any object with the same
    attributes: stun_host, stun_port, turn_host, turn_port, turn_protocol, turn_tls,
    turn_shared_secret, turn_username, turn_password)."""
    servers: list[dict] = []
    if getattr(cfg, "stun_host", None):
        servers.append({"urls": [f"stun:{cfg.stun_host}:{cfg.stun_port}"]})
    if getattr(cfg, "turn_host", None):
        urls = turn_urls(cfg.turn_host, int(cfg.turn_port), cfg.turn_protocol or "udp", bool(cfg.turn_tls))
        if getattr(cfg, "turn_shared_secret", None):
            u, p = hmac_credentials(cfg.turn_shared_secret, user, now=now)
            servers.append({"urls": urls, "username": u, "credential": p})
        elif getattr(cfg, "turn_username", None) and getattr(cfg, "turn_password", None):
            servers.append({"urls": urls, "username": cfg.turn_username, "credential": cfg.turn_password})
        else:
            servers.append({"urls": urls})
    return {"lifetimeDuration": "86400s", "iceServers": servers, "blockStatus": "NOT_BLOCKED",
            "iceTransportPolicy": "all"}


async def fetch_rest_credentials(uri: str, username: str = "mxdesk", protocol: str = "udp", tls: bool = False,
                                 timeout: float = 5.0) -> dict:
    """GET a TURN REST URI (selkies-compatible headers) and return its RTC config JSON."""
    import aiohttp

    headers = {"x-auth-user": username, "x-turn-protocol": protocol, "x-turn-tls": str(tls).lower()}
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout)) as s:
        async with s.get(uri, headers=headers) as r:
            r.raise_for_status()
            return json.loads(await r.text())
