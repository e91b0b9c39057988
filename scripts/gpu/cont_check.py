import sys, time, torch
sys.path.insert(0, ".")
from pretraining_llm_amd.inference.server import ContinuousGenerationServer, GenRequest
from pretraining_llm_amd.models import GPT, get_preset
from pretraining_llm_amd.ops import _lib
_lib.require()
torch.manual_seed(0)
dev = torch.device("cuda", 0)
model = GPT(get_preset("gpt2-small")).to(device=dev, dtype=torch.bfloat16).eval()
g = torch.Generator().manual_seed(1)
prompts = [torch.randint(0, 50304, (int(n),), generator=g).tolist() for n in torch.randint(8, 64, (16,), generator=g)]
cs = ContinuousGenerationServer(model, max_batch=16, max_len=200)
res = [f.result() for f in [cs.submit(GenRequest(p, max_new_tokens=24, temperature=0.0)) for p in prompts]]
cs.close()
# reference: the same prompts through lockstep batched generate, one prompt-length group at a time (B=1 each)
agree = 0
for p, r in zip(prompts, res):
    ref = model.generate(torch.tensor([p], device=dev), max_new_tokens=24, temperature=0.0, cuda_graph=True)[0].tolist()
    n = next((i for i, (a, b) in enumerate(zip(r.tokens[len(p):], ref[len(p):])) if a != b), 24)
    agree += n
    print(len(p), "first divergence at new token", n, "latency", round(r.latency_ms, 1), "batch", r.batch_size)
print("mean agreeing prefix", agree / len(prompts))
