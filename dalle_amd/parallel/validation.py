"""Record validators for the DHT facade (``utils.py:23-30``: SchemaValidator + RSASignatureValidator).

* :class:`SchemaValidator` validates records whose key is ``{prefix}_{field}`` against the pydantic
  schema's field type (``MetricSchema{metrics: Dict[BytesWithPublicKey, LocalMetrics]}``).
* :class:`RSASignatureValidator` gives every peer an owner identity (``local_public_key``). There is
  no asymmetric-crypto library in this image, so ownership is enforced by the native store itself:
  a live subkey can only be rewritten by the owner that created it (csrc/store/kvstore.cpp).
"""
from __future__ import annotations

import secrets
from typing import Any, Dict

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
    def __init__(self, local_public_key: bytes = None):
        self.local_public_key = local_public_key or (b"<rsa-pubkey:" + secrets.token_hex(16).encode() + b">")

    def validate(self, key: str, subkey: Any, value: Any) -> bool:
        return True
