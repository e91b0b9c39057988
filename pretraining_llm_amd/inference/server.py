"""Batched generation service (HTTP) over the KV-cache decoder.

The reference serves text only through a one-shot CLI (scripts/generate_text.py:7-61: load,
generate one prompt, exit).  For serving, the model stays resident and concurrent requests are
batched: a worker thread drains a request queue, waits up to ``max_wait_ms`` for company, groups
requests that can share one decode batch -- same prompt length and the same sampling settings,
since every sequence of a batch advances through the same cache positions -- and runs each group
as ONE batched ``generate`` (prefill through the flash-attention kernel, then one hipGraph replay
per token, csrc/attn_decode.hip + csrc/gemv.hip + csrc/sampling.hip on the GPU).  Decode at batch
64 is ~24x the tokens/s of batch 1 (README, profiles/r1_decode_bench_fused.jsonl), so batching is
where serving throughput comes from.

``GenerationServer`` (lockstep groups) and ``ContinuousGenerationServer`` (continuous batching:
decode slots at per-sequence positions, requests join and leave the running batch one token step
at a time) are usable in-process (``submit`` -> Future); ``create_app`` wraps either in a FastAPI
app (POST /generate, GET /health, GET /stats); ``scripts/serve.py`` runs it under uvicorn.
"""

import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch


@dataclass
class GenRequest:
    tokens: List[int]
    max_new_tokens: int = 64
    temperature: float = 1.0
    top_k: Optional[int] = None
    seed: Optional[int] = None
    t_submit: float = field(default_factory=time.perf_counter)

    def group_key(self):
        # sequences decode in lockstep: one prompt length, one number of steps, one sampler.  A
        # seeded request is never batched with another: its tokens must not depend on its row or
        # on its batch-mates, so it decodes alone with its own generator (= single-request generate)
        private = id(self) if self.seed is not None else None
        return (len(self.tokens), self.max_new_tokens, float(self.temperature), self.top_k, self.seed, private)


@dataclass
class GenResult:
    tokens: List[int]          # prompt + generated ids
    new_tokens: List[int]      # generated ids only
    batch_size: int            # how many requests shared the decode batch
    latency_ms: float          # submit -> result


class GenerationServer:
    def __init__(self, model, max_batch: int = 64, max_wait_ms: float = 5.0, cuda_graph: bool = True,
                 max_cached_shapes: int = 16):
        self.model = model.eval()
        self.device = next(model.parameters()).device
        self.max_batch = int(max_batch)
        self.max_wait = max_wait_ms / 1e3
        self.max_cached_shapes = int(max_cached_shapes)
        self.cuda_graph = cuda_graph and self.device.type == "cuda"
        self._q = queue.Queue()
        self._decode_cache = {}  # (batch, cache length) -> KV cache + captured decode graph, reused
        self._stop = threading.Event()
        self._submit_lock = threading.Lock()
        self.stats: Dict[str, float] = {"requests": 0, "batches": 0, "generated_tokens": 0, "max_batch_seen": 0}
        self._worker = threading.Thread(target=self._run, name="pllm-generation", daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------
    def submit(self, req: GenRequest) -> Future:
        ctx = self.model.config.context_length
        if not req.tokens:
            raise ValueError("empty prompt")
        if req.max_new_tokens < 1:
            raise ValueError("max_new_tokens must be >= 1")
        if any(t < 0 or t >= self.model.config.vocab_size for t in req.tokens):
            raise ValueError("token id outside the vocabulary")
        if self.model.config.pos != "learned" and len(req.tokens) + req.max_new_tokens > 8 * ctx:
            raise ValueError("prompt + max_new_tokens too long")
        fut: Future = Future()
        with self._submit_lock:  # no request can be queued behind close()'s stop marker
            if self._stop.is_set():
                raise RuntimeError("generation server closed")
            self._q.put((req, fut))
        return fut

    def close(self):
        with self._submit_lock:
            self._stop.set()
            self._q.put(None)
        self._worker.join(timeout=30)
        while True:  # requests still queued behind the stop marker fail instead of waiting forever
            try:
                it = self._q.get_nowait()
            except queue.Empty:
                break
            if it is not None:
                it[1].set_exception(RuntimeError("generation server closed"))

    # ------------------------------------------------------------------
    def _collect(self):
        first = self._q.get()
        if first is None:
            return None
        items = [first]
        deadline = time.perf_counter() + self.max_wait
        while len(items) < self.max_batch:
            left = deadline - time.perf_counter()
            if left <= 0:
                break
            try:
                it = self._q.get(timeout=left)
            except queue.Empty:
                break
            if it is None:
                self._stop.set()
                break
            items.append(it)
        return items

    def _run(self):
        while not self._stop.is_set():
            items = self._collect()
            if items is None:
                return
            groups: Dict[tuple, list] = {}
            for req, fut in items:
                groups.setdefault(req.group_key(), []).append((req, fut))
            for key, members in groups.items():
                for i in range(0, len(members), self.max_batch):
                    self._serve(members[i:i + self.max_batch])

    def _serve(self, members):
        req0 = members[0][0]
        try:
            idx = torch.tensor([r.tokens for r, _ in members], dtype=torch.long, device=self.device)
            gen = None
            if req0.seed is not None:
                gen = torch.Generator(device=self.device).manual_seed(int(req0.seed))
            with torch.no_grad():
                out = self.model.generate(idx, max_new_tokens=req0.max_new_tokens, temperature=req0.temperature,
                                          top_k=req0.top_k, generator=gen, cuda_graph=self.cuda_graph,
                                          decode_cache=self._decode_cache)
            out = out.tolist()
            while len(self._decode_cache) > self.max_cached_shapes:  # oldest shape first
                self._decode_cache.pop(next(iter(self._decode_cache)))
        except Exception as e:  # deliver the failure to every waiter of the batch
            for _, fut in members:
                fut.set_exception(e)
            return
        now = time.perf_counter()
        n = len(members)
        self.stats["requests"] += n
        self.stats["batches"] += 1
        self.stats["generated_tokens"] += n * req0.max_new_tokens
        self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], n)
        for (r, fut), seq in zip(members, out):
            fut.set_result(GenResult(tokens=seq, new_tokens=seq[len(r.tokens):], batch_size=n,
                                     latency_ms=1e3 * (now - r.t_submit)))


def create_app(server: GenerationServer, tokenizer=None):
    """FastAPI app: POST /generate {prompt | tokens, max_new_tokens, temperature, top_k, seed},
    GET /health, GET /stats."""
    import asyncio

    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    class GenerateBody(BaseModel):
        prompt: Optional[str] = None
        tokens: Optional[List[int]] = None
        max_new_tokens: int = 64
        temperature: float = 1.0
        top_k: Optional[int] = None
        seed: Optional[int] = None

    app = FastAPI(title="pretraining-llm-amd generation")
    cfg = server.model.config

    @app.get("/health")
    def health():
        return {"status": "ok", "device": str(server.device), "arch": cfg.arch, "n_blocks": cfg.n_blocks,
                "n_embed": cfg.n_embed, "vocab_size": cfg.vocab_size, "context_length": cfg.context_length}

    @app.get("/stats")
    def stats():
        return dict(server.stats)

    @app.post("/generate")
    async def generate(body: GenerateBody):
        if body.tokens is None and body.prompt is None:
            raise HTTPException(400, "give 'prompt' or 'tokens'")
        if body.tokens is not None:
            toks = list(body.tokens)
        else:
            if tokenizer is None:
                raise HTTPException(400, "no tokenizer loaded: send 'tokens'")
            toks = tokenizer.encode_ordinary(body.prompt) or [tokenizer.eot_token % cfg.vocab_size]
        try:
            fut = server.submit(GenRequest(toks, body.max_new_tokens, body.temperature, body.top_k, body.seed))
        except ValueError as e:
            raise HTTPException(400, str(e))
        res: GenResult = await asyncio.wrap_future(fut)
        out = {"tokens": res.new_tokens, "prompt_tokens": len(toks), "batch_size": res.batch_size,
               "latency_ms": round(res.latency_ms, 3)}
        if tokenizer is not None:
            out["text"] = tokenizer.decode(res.tokens)
        return out

    return app


class ContinuousGenerationServer:
    """Continuous batching: a fixed set of ``max_batch`` decode slots, each sequence at its own
    position.  A request is prefilled alone into a free slot (flash attention over its prompt)
    as soon as one frees up, then joins the shared decode step: one step advances every active
    slot by one token (per-sequence positions and key counts go to the decode kernels as device
    tensors -- csrc/attn_decode.hip, csrc/gemv.hip -- so the step is one hipGraph replay for the
    whole slot set), and a finished sequence leaves without waiting for the others.  Unlike the
    lockstep ``GenerationServer`` no request waits for company of the same prompt length.

    Learned absolute positions (arch ref / gpt2) follow the reference's crop semantics: a slot
    whose sequence reaches ``context_length`` is re-prefilled on its last ``context_length``
    tokens for every further token (transformer.py:108), outside the shared step."""

    def __init__(self, model, max_batch: int = 32, max_len: Optional[int] = None, cuda_graph: bool = True):
        from .generate import DecodeGraph, KVCache
        cfg = model.config
        self.model = model.eval()
        self.device = next(model.parameters()).device
        self.B = int(max_batch)
        self.learned = cfg.pos == "learned"
        self.ctx = cfg.context_length
        self.max_len = self.ctx if self.learned else int(max_len or self.ctx)
        dtype = model.token_embed.weight.dtype
        self.cache = KVCache(cfg.n_blocks, self.B, self.max_len, cfg.n_kv_head, cfg.head_dim, dtype, self.device)
        self.graph = None
        if cuda_graph and self.device.type == "cuda":
            # captured before any prefill: its warm-up steps write cache row 0 of every slot,
            # which a slot's prefill overwrites before the slot is used
            self.graph = DecodeGraph(model, self.cache, self.B, self.device, per_row=True)
        self.slots: List[Optional[dict]] = [None] * self.B
        # device-resident decode state: the next input token of every slot and each slot's
        # generated tokens, so a decode step needs no host <-> device round trip
        self.tok_d = torch.zeros(self.B, 1, dtype=torch.long, device=self.device)
        self.out_d = torch.zeros(self.B, 256, dtype=torch.long, device=self.device)
        self._q = queue.Queue()
        self._stop = threading.Event()
        self._submit_lock = threading.Lock()
        self.stats: Dict[str, float] = {"requests": 0, "decode_steps": 0, "generated_tokens": 0,
                                        "max_active_slots": 0, "prefills": 0}
        self._worker = threading.Thread(target=self._run, name="pllm-continuous-batching", daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------ API (as GenerationServer)
    def submit(self, req: GenRequest) -> Future:
        if not req.tokens:
            raise ValueError("empty prompt")
        if req.max_new_tokens < 1:
            raise ValueError("max_new_tokens must be >= 1")
        if any(t < 0 or t >= self.model.config.vocab_size for t in req.tokens):
            raise ValueError("token id outside the vocabulary")
        if not self.learned and len(req.tokens) + req.max_new_tokens > self.max_len:
            raise ValueError(f"prompt + max_new_tokens exceeds the server's cache length {self.max_len}")
        fut: Future = Future()
        with self._submit_lock:
            if self._stop.is_set():
                raise RuntimeError("generation server closed")
            self._q.put((req, fut))
        return fut

    def close(self):
        with self._submit_lock:
            self._stop.set()
            self._q.put(None)
        self._worker.join(timeout=60)
        while True:
            try:
                it = self._q.get_nowait()
            except queue.Empty:
                break
            if it is not None:
                it[1].set_exception(RuntimeError("generation server closed"))

    # ------------------------------------------------------------------ internals
    def _slot_cache(self, s: int):
        from .generate import KVCache
        view = KVCache.__new__(KVCache)
        view.k = [t[s:s + 1] for t in self.cache.k]
        view.v = [t[s:s + 1] for t in self.cache.v]
        view.max_len = self.max_len
        return view

    def _prefill_batch(self, slots: List[int], prompts: List[List[int]]) -> torch.Tensor:
        """Prefill several requests in ONE forward: prompts right-padded to the longest (causal
        attention keeps real tokens blind to the padding behind them; the padded K/V rows sit past
        each slot's key count and are overwritten by its decode steps), run into a temporary cache
        and scattered into the slots' cache rows.  Returns the logits at each prompt's last token."""
        from .generate import KVCache, forward_cached
        T = max(len(p) for p in prompts)
        n = len(prompts)
        idx = torch.zeros(n, T, dtype=torch.long)
        for i, p in enumerate(prompts):
            idx[i, :len(p)] = torch.tensor(p, dtype=torch.long)
        last = torch.tensor([len(p) - 1 for p in prompts], dtype=torch.long, device=self.device)
        cfg = self.model.config
        tmp = KVCache(cfg.n_blocks, n, T, cfg.n_kv_head, cfg.head_dim, self.cache.k[0].dtype, self.device)
        self.stats["prefills"] += 1
        with torch.no_grad():
            logits = forward_cached(self.model, idx.to(self.device), tmp, 0, last=last)
            sl = torch.tensor(slots, dtype=torch.long, device=self.device)
            for layer in range(cfg.n_blocks):
                self.cache.k[layer][sl, :T] = tmp.k[layer]
                self.cache.v[layer][sl, :T] = tmp.v[layer]
        return logits

    def _prefill(self, s: int, tokens: List[int]) -> torch.Tensor:
        from .generate import forward_cached
        window = tokens[-self.ctx:] if self.learned else tokens
        idx = torch.tensor([window], dtype=torch.long, device=self.device)
        self.stats["prefills"] += 1
        with torch.no_grad():
            return forward_cached(self.model, idx, self._slot_cache(s), 0), len(window)

    def _sample(self, rows: List[int], logits: torch.Tensor) -> torch.Tensor:
        """Next token for each slot in ``rows`` (logits row k belongs to slot rows[k]) as a device
        int64 [len(rows)] tensor (no host sync); slots with the same sampler and no private seed
        share one fused sampling launch."""
        from .generate import sample_next
        groups: Dict[tuple, List[int]] = {}
        for k, s in enumerate(rows):
            r = self.slots[s]["req"]
            key = (float(r.temperature), r.top_k, s if r.seed is not None else -1)
            groups.setdefault(key, []).append(k)
        if len(groups) == 1:
            (temp, top_k, private), = groups.keys()
            gen = self.slots[rows[0]]["gen"] if private >= 0 else None
            return sample_next(logits, temp, top_k, gen).view(-1)
        out = torch.empty(len(rows), dtype=torch.long, device=logits.device)
        for (temp, top_k, private), ks in groups.items():
            gen = self.slots[rows[ks[0]]]["gen"] if private >= 0 else None
            idx = self._dev_index(ks)
            out.index_copy_(0, idx, sample_next(logits.index_select(0, idx), temp, top_k, gen).view(-1))
        return out

    def _dev_index(self, values: List[int]) -> torch.Tensor:
        # small index lists go through pinned memory with an async copy: no host <-> device sync
        h = torch.tensor(values, dtype=torch.long).pin_memory() if self.device.type == "cuda" else \
            torch.tensor(values, dtype=torch.long)
        return h.to(self.device, non_blocking=True)

    def _record(self, rows: List[int], toks: torch.Tensor):
        """Append the sampled tokens of ``rows`` on the device: the decode input buffer and each
        slot's output row (read back to the host once, when the request finishes)."""
        idx = self._dev_index(rows)
        cols = self._dev_index([self.slots[s]["n_new"] for s in rows])
        self.tok_d.index_copy_(0, idx, toks.view(-1, 1))
        self.out_d.index_put_((idx, cols), toks.view(-1))
        for s in rows:
            self.slots[s]["n_new"] += 1

    def _finish_done(self):
        done = [s for s, sl in enumerate(self.slots)
                if sl is not None and sl["n_new"] >= sl["req"].max_new_tokens]
        if not done:
            return
        outs = self.out_d[self._dev_index(done)].tolist()  # the one host sync per finished batch of requests
        # stamped AFTER the read-back: decode steps are enqueued asynchronously, so only the sync
        # above says the tokens exist (a stamp before it measured host enqueue time)
        now = time.perf_counter()
        for s, row in zip(done, outs):
            sl = self.slots[s]
            r = sl["req"]
            new = row[:r.max_new_tokens]
            self.stats["requests"] += 1
            self.stats["generated_tokens"] += r.max_new_tokens
            sl["fut"].set_result(GenResult(tokens=list(r.tokens) + new, new_tokens=new, batch_size=sl["peak_batch"],
                                           latency_ms=1e3 * (now - r.t_submit)))
            self.slots[s] = None

    def _admit(self, block: bool):
        admitted = []
        while any(sl is None for sl in self.slots):
            try:
                it = self._q.get(timeout=0.05) if block else self._q.get_nowait()
            except queue.Empty:
                break
            block = False
            if it is None:
                self._stop.set()
                break
            req, fut = it
            s = self.slots.index(None)
            try:
                gen = None
                if req.seed is not None:
                    gen = torch.Generator(device=self.device).manual_seed(int(req.seed))
                if req.max_new_tokens > self.out_d.shape[1]:
                    self._grow_out(req.max_new_tokens)
                window = req.tokens[-self.ctx:] if self.learned else req.tokens
                self.slots[s] = {"req": req, "fut": fut, "pos": len(window), "n_new": 0, "gen": gen,
                                 "peak_batch": 1, "window": window}
                admitted.append(s)
            except Exception as e:  # a bad request fails alone
                self.slots[s] = None
                fut.set_exception(e)
        # prefill the newly admitted requests together, in batches of similar length (right padding
        # wastes at most PREFILL_PAD_FRACTION of a batch's tokens)
        admitted.sort(key=lambda s: len(self.slots[s]["window"]))
        i = 0
        while i < len(admitted):
            j = i + 1
            while j < len(admitted):
                L = len(self.slots[admitted[j]]["window"])
                real = sum(len(self.slots[s]["window"]) for s in admitted[i:j + 1])
                if real < (1.0 - self.PREFILL_PAD_FRACTION) * L * (j + 1 - i):
                    break
                j += 1
            group = admitted[i:j]
            try:
                logits = self._prefill_batch(group, [self.slots[s]["window"] for s in group])
                self._record(group, self._sample(group, logits))
            except Exception as e:
                for s in group:
                    self.slots[s]["fut"].set_exception(e)
                    self.slots[s] = None
            i = j
        self._finish_done()

    PREFILL_PAD_FRACTION = 0.25

    def _grow_out(self, n: int):
        out = torch.zeros(self.B, n, dtype=torch.long, device=self.device)
        out[:, :self.out_d.shape[1]] = self.out_d
        self.out_d = out

    def _history(self, s: int) -> List[int]:
        sl = self.slots[s]
        return list(sl["req"].tokens) + self.out_d[s, :sl["n_new"]].tolist()

    def _step(self):
        from .generate import forward_decode
        active = [s for s, sl in enumerate(self.slots) if sl is not None]
        if not active:
            return
        self.stats["max_active_slots"] = max(self.stats["max_active_slots"], len(active))
        for s in active:
            self.slots[s]["peak_batch"] = max(self.slots[s]["peak_batch"], len(active))
        shared = []
        for s in active:
            sl = self.slots[s]
            if self.learned and sl["pos"] >= self.ctx:  # crop semantics: re-prefill the last ctx tokens
                logits, sl["pos"] = self._prefill(s, self._history(s))
                self._record([s], self._sample([s], logits))
            else:
                shared.append(s)
        if shared:
            pos = [0] * self.B  # idle slots decode a dummy token at row 0 (overwritten by their next prefill)
            for s in shared:
                pos[s] = self.slots[s]["pos"]
            pos_t = self._dev_index(pos)
            with torch.no_grad():
                if self.graph is not None:
                    logits = self.graph(self.tok_d, pos_t)
                else:
                    logits = forward_decode(self.model, self.tok_d, self.cache, pos_t, (pos_t + 1).to(torch.int32))
            sel = logits if len(shared) == self.B else logits.index_select(0, self._dev_index(shared))
            self._record(shared, self._sample(shared, sel))
            for s in shared:
                self.slots[s]["pos"] += 1
            self.stats["decode_steps"] += 1
        self._finish_done()

    def _run(self):
        while not self._stop.is_set():
            try:
                self._admit(block=all(sl is None for sl in self.slots))
                self._step()
            except Exception as e:  # fail every in-flight request rather than hang them
                for s, sl in enumerate(self.slots):
                    if sl is not None:
                        sl["fut"].set_exception(e)
                        self.slots[s] = None
        for s, sl in enumerate(self.slots):
            if sl is not None:
                sl["fut"].set_exception(RuntimeError("generation server closed"))
                self.slots[s] = None
