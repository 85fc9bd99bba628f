"""JWT (HS256) tokens, password hashing and role-based access control.

Reference parity: rafiki/utils/auth.py (:10-59: 1 h tokens, ``auth(user_types)`` decorator with
SUPERADMIN always allowed, ``Bearer`` header parsing) and bcrypt hashing in admin.py:635-640.
PyJWT and bcrypt are not available offline; HS256 is implemented with ``hmac``/``hashlib`` and
passwords use ``hashlib.scrypt`` (memory-hard, salted).  Fixes reference bug (h): ``auth()`` no
longer mutates a shared default list.
"""
from __future__ import annotations

import base64
import functools
import hashlib
import hmac
import json
import os
import time

from ..constants import UserType

TOKEN_EXPIRATION_HOURS = 1


class UnauthorizedError(Exception):
    pass


class InvalidAuthorizationHeaderError(Exception):
    pass


def _b64e(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b'=').decode('ascii')


def _b64d(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + '=' * (-len(s) % 4))


def _secret():
    from .. import config
    return config.APP_SECRET.encode('utf-8')


def generate_token(user, expiration_hours=TOKEN_EXPIRATION_HOURS):
    """``user`` is a dict with ``user_id`` and ``user_type``."""
    header = {'alg': 'HS256', 'typ': 'JWT'}
    payload = dict(user)
    payload['exp'] = int(time.time() + expiration_hours * 3600)
    seg = _b64e(json.dumps(header, separators=(',', ':')).encode()) + '.' + \
        _b64e(json.dumps(payload, separators=(',', ':'), default=str).encode())
    sig = hmac.new(_secret(), seg.encode('ascii'), hashlib.sha256).digest()
    return seg + '.' + _b64e(sig)


def decode_token(token):
    try:
        h, p, s = token.split('.')
    except (ValueError, AttributeError):
        raise UnauthorizedError('malformed token')
    expect = hmac.new(_secret(), (h + '.' + p).encode('ascii'), hashlib.sha256).digest()
    if not hmac.compare_digest(expect, _b64d(s)):
        raise UnauthorizedError('bad token signature')
    payload = json.loads(_b64d(p))
    if payload.get('exp', 0) < time.time():
        raise UnauthorizedError('token expired')
    return payload


def hash_password(password: str) -> bytes:
    salt = os.urandom(16)
    dk = hashlib.scrypt(password.encode('utf-8'), salt=salt, n=2 ** 12, r=8, p=1, dklen=32)
    return b'scrypt$' + base64.b64encode(salt) + b'$' + base64.b64encode(dk)


def check_password(password: str, stored: bytes) -> bool:
    if isinstance(stored, str):
        stored = stored.encode('utf-8')
    try:
        _, salt_b64, dk_b64 = stored.split(b'$')
    except ValueError:
        return False
    dk = hashlib.scrypt(password.encode('utf-8'), salt=base64.b64decode(salt_b64), n=2 ** 12, r=8, p=1, dklen=32)
    return hmac.compare_digest(dk, base64.b64decode(dk_b64))


def extract_token_from_header(header):
    if header is None:
        raise InvalidAuthorizationHeaderError()
    parts = header.split(' ')
    if len(parts) != 2 or parts[0] != 'Bearer':
        raise InvalidAuthorizationHeaderError()
    return parts[1]


def auth(user_types=None):
    """Flask route decorator: injects ``auth`` (decoded token) as the first arg; SUPERADMIN always passes."""
    allowed = set(user_types or []) | {UserType.SUPERADMIN}

    def decorator(f):
        @functools.wraps(f)
        def wrapped(*args, **kwargs):
            from flask import request
            try:
                token = extract_token_from_header(request.headers.get('authorization'))
                payload = decode_token(token)
            except (InvalidAuthorizationHeaderError, UnauthorizedError):
                return 'Unauthorized', 401
            if payload.get('user_type') not in allowed:
                return 'Forbidden', 403
            return f(payload, *args, **kwargs)
        return wrapped
    return decorator
