"""Record validators for the DHT facade (``utils.py:23-30``: SchemaValidator + RSASignatureValidator).

* :class:`SchemaValidator` validates records whose key is ``{prefix}_{field}`` against the pydantic
  schema's field type (``MetricSchema{metrics: Dict[BytesWithPublicKey, LocalMetrics]}``).
* :class:`RSASignatureValidator` gives every peer an RSA owner identity (``local_public_key``) and
  signs / verifies owner-protected records (``dalle_amd.parallel.crypto``). The native store also
  refuses to let anyone but a live subkey's creator rewrite it (csrc/store/kvstore.cpp).
"""
from __future__ import annotations

import base64
import re
from typing import Any, Dict

import msgpack

BytesWithPublicKey = bytes


class RecordValidatorBase:
    def validate(self, key: str, subkey: Any, value: Any) -> bool:  # pragma: no cover - interface
        return True


class SchemaValidator(RecordValidatorBase):
    def __init__(self, schema, prefix: str = None, allow_extra_keys: bool = True):
        self.schema = schema
        self.prefix = prefix
        self.allow_extra_keys = allow_extra_keys
        fields = getattr(schema, "model_fields", None) or getattr(schema, "__fields__", {})
        self.fields = dict(fields)

    def _field_of(self, key: str):
        if self.prefix is not None:
            if not key.startswith(self.prefix + "_"):
                return None
            key = key[len(self.prefix) + 1:]
        return key if key in self.fields else None

    def validate(self, key: str, subkey: Any, value: Any) -> bool:
        field = self._field_of(key)
        if field is None:
            return self.allow_extra_keys
        try:
            payload: Dict[str, Any] = {field: {subkey: value} if subkey is not None else value}
            if hasattr(self.schema, "model_validate"):
                self.schema.model_validate(payload)
            else:
                self.schema.parse_obj(payload)
            return True
        except Exception:
            return False


class RSASignatureValidator(RecordValidatorBase):
    """Owner-signed records (hivemind ``RSASignatureValidator`` semantics).

    ``local_public_key`` is ``[owner:<ssh-rsa public key>]``. A record whose key or subkey contains an
    owner marker must carry exactly one ``[signature:<base64>]`` suffix in its serialised value: an
    RSASSA-PKCS1-v1_5 / SHA-256 signature by that owner over ``msgpack([key, subkey, value,
    expiration_time])`` with the signature stripped. Unprotected records pass unchanged. The DHT
    facade signs on store and validates + strips on every read, so a record forged by another peer
    (or altered in the store) never reaches a consumer.
    """

    PUBLIC_KEY_FORMAT = b"[owner:_key_]"
    SIGNATURE_FORMAT = b"[signature:_value_]"
    _PUBLIC_KEY_RE = re.compile(rb"\[owner:(.+?)\]")
    _SIGNATURE_RE = re.compile(rb"\[signature:(.+?)\]")

    def __init__(self, private_key=None):
        from .crypto import RSAPrivateKey

        self._private_key = private_key or RSAPrivateKey.process_wide()
        self.local_public_key = self.PUBLIC_KEY_FORMAT.replace(b"_key_", self._private_key.get_public_key().to_bytes())

    @staticmethod
    def _as_bytes(x) -> bytes:
        if x is None:
            return b""
        return x if isinstance(x, bytes) else str(x).encode()

    def _serialize(self, key, subkey, value: bytes, expiration_time: float) -> bytes:
        return msgpack.packb([self._as_bytes(key), self._as_bytes(subkey), value, float(expiration_time)], use_bin_type=True)

    def sign_value(self, key, subkey, value: bytes, expiration_time: float) -> bytes:
        if self.local_public_key not in self._as_bytes(key) and self.local_public_key not in self._as_bytes(subkey):
            return value
        sig = self._private_key.sign(self._serialize(key, subkey, value, expiration_time))
        return value + self.SIGNATURE_FORMAT.replace(b"_value_", base64.b64encode(sig))

    def strip_value(self, value: bytes) -> bytes:
        return self._SIGNATURE_RE.sub(b"", value)

    def validate_signed(self, key, subkey, value: bytes, expiration_time: float) -> bool:
        from .crypto import RSAPublicKey

        keys = self._PUBLIC_KEY_RE.findall(self._as_bytes(key)) + self._PUBLIC_KEY_RE.findall(self._as_bytes(subkey))
        if not keys:
            return True  # not owner-protected
        if len(set(keys)) > 1:
            return False
        sigs = self._SIGNATURE_RE.findall(value)
        if len(sigs) != 1:
            return False
        try:
            pub = RSAPublicKey.from_bytes(keys[0])
            return pub.verify(self._serialize(key, subkey, self.strip_value(value), expiration_time), base64.b64decode(sigs[0]))
        except Exception:  # malformed key / signature
            return False

    def validate(self, key: str, subkey: Any, value: Any) -> bool:
        return True  # ownership is checked on the serialised record (validate_signed)
