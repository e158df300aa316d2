"""`web_api` run mode: FastAPI routes with the reference's names and schemas (ref src/rest_api.py:13-89).

Routes (all POST): ``/check_tokens``, ``/encode``, ``/decode``, ``/token_completion``, ``/completion``.
Bug A15 is fixed: ``decode`` decodes (the reference calls ``encode``). The server runs in a thread of the GPU
process (no Manager-dict IPC); requests are batched by ``CompletionEngine``.
"""
from __future__ import annotations

import asyncio
import threading
import typing

from ..config import ModelParameter
from .infer import CompletionEngine, ContextExhaustedError, InvalidTokenError, Tokenizer

try:
    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel
except ImportError:  # pragma: no cover - fastapi is part of the image
    FastAPI = None


if FastAPI is not None:
    class Tokens(BaseModel):
        tokens: typing.List[int]

    class TokenCompletion(BaseModel):
        token_completion: typing.List[int]

    class Completion(BaseModel):
        completion: str

    class SanitizedTokens(BaseModel):
        tokens: typing.List[int]

    class CompletionInput(BaseModel):
        prompt: str = ""
        max_tokens: int = 16
        temperature: float = 1.
        error: bool = True


class RestAPI:
    def __init__(self, engine: CompletionEngine, tokenizer: Tokenizer, params: ModelParameter):
        self._engine, self._tok, self._params = engine, tokenizer, params

    async def check_tokens(self, tokens: typing.List[int], error: bool = True) -> "SanitizedTokens":
        p = self._params
        if tokens and max(tokens) >= p.vocab_size:
            if error:
                raise HTTPException(status_code=400, detail=f"Invalid tokens sent. Tokens go up to "
                                                            f"{p.vocab_size - 1} but received {max(tokens)}.")
            tokens = [t for t in tokens if t < p.vocab_size]
        if len(tokens) > p.sequence_length:
            if error:
                raise HTTPException(status_code=400, detail=f"Context too big. The model supports up to "
                                                            f"{p.sequence_length} tokens but received {len(tokens)}.")
            tokens = tokens[:p.sequence_length]
        return SanitizedTokens(tokens=tokens)

    async def encode(self, prompt: str) -> "Tokens":
        return Tokens(tokens=self._tok.encode(prompt))

    async def decode(self, prompt: typing.List[int]) -> "Completion":
        return Completion(completion=self._tok.decode(prompt))

    async def token_completion(self, params: "CompletionInput") -> "TokenCompletion":
        tokens = (await self.encode(params.prompt)).tokens
        tokens = (await self.check_tokens(tokens, params.error)).tokens
        fut = self._engine.submit(tokens, params.temperature, len(tokens) + params.max_tokens) \
            if len(tokens) < self._params.sequence_length else None
        if fut is None:
            raise HTTPException(status_code=400, detail="no room left in the context")
        out = await asyncio.get_running_loop().run_in_executor(None, fut.get)
        if isinstance(out, (ContextExhaustedError, InvalidTokenError)):
            raise HTTPException(status_code=400, detail=str(out))
        if isinstance(out, BaseException):
            raise HTTPException(status_code=500, detail=repr(out))
        return TokenCompletion(token_completion=out.tolist()[:params.max_tokens])

    async def completion(self, params: "CompletionInput") -> "Completion":
        return await self.decode((await self.token_completion(params)).token_completion)


def build_app(api: RestAPI):
    if FastAPI is None:
        raise RuntimeError("fastapi is not importable")
    app = FastAPI()
    for key in ("check_tokens", "encode", "decode", "token_completion", "completion"):
        fn = getattr(api, key)
        app.post("/" + key, response_model=typing.get_type_hints(fn)["return"])(fn)
    return app


def serve(api: RestAPI, host: str, port: int, workers: int = 1) -> threading.Thread:
    """uvicorn in a background thread of this process (one GPU owner, many HTTP clients)"""
    import uvicorn
    config = uvicorn.Config(build_app(api), host=host, port=port, log_level="info", workers=workers)
    server = uvicorn.Server(config)
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    t.server = server  # type: ignore[attr-defined]
    return t
