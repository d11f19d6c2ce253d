"""HTTP Basic authentication (reference Dockerfile:212 ENABLE_BASIC_AUTH,
selkies-gstreamer-entrypoint.sh:20 BASIC_AUTH_PASSWORD defaulting to PASSWD; user name
``user``, README.md:23)."""
from __future__ import annotations

import base64
import hmac

from aiohttp import web

PUBLIC_PATHS = ("/health",)


def check_basic(header: str | None, user: str, password: str) -> bool:
    if not header or not header.startswith("Basic "):
        return False
    try:
        raw = base64.b64decode(header[6:].strip(), validate=True).decode("utf-8")
    except (ValueError, UnicodeDecodeError):
        return False
    u, sep, p = raw.partition(":")
    if not sep:
        return False
    # constant-time comparisons (both evaluated)
    ok_u = hmac.compare_digest(u.encode(), user.encode())
    ok_p = hmac.compare_digest(p.encode(), password.encode())
    return ok_u and ok_p


def basic_auth_middleware(user: str, password: str, realm: str = "mxdesk"):
    @web.middleware
    async def mw(request: web.Request, handler):
        if request.path in PUBLIC_PATHS or check_basic(request.headers.get("Authorization"), user, password):
            return await handler(request)
        return web.Response(status=401, headers={"WWW-Authenticate": f'Basic realm="{realm}", charset="UTF-8"'},
                            text="401: Unauthorized")

    return mw
