"""diagnostic: first-layer weight-gradient error of the fused engine vs fp32 torch, by schedule knobs"""
import os, sys, json, subprocess
code = r'''
import sys, torch, torch.nn.functional as F, json
sys.path.insert(0, "/root/repo")
from neural_net_model import NeuralNetworkModel
from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
sizes = [1024, 4096, 4096, 1024]; n, S, lr, l2 = 16384, 8192, 0.01, 1e-3
torch.manual_seed(3)
model = NeuralNetworkModel("m", sizes, "xavier", "random", ["relu", "relu", "softmax"], "stochastic", dtype="bfloat16", device="cuda")
g = torch.Generator().manual_seed(8)
inputs = torch.randn(n, sizes[0], generator=g); labels = torch.randint(0, sizes[-1], (n,), generator=g)
tr = FusedTrainer(model); tr.load_tensors(inputs, labels, seed=5); tr.begin(1)
p0 = [p.detach().float().clone() for p in model.params]
tr.step(0, lr, S, 0.0, l2, want_ratios=True, record=False); tr.drain()
picked = tr.picked[:S].clone(); p1 = [p.detach().float().clone() for p in model.params]
ref = [p.clone().requires_grad_() for p in p0]; w1, b1, w2, b2, w3, b3 = ref
x = tr.data[picked].float(); y = labels.to(x.device)[picked]
h = torch.relu(x @ w1 + b1); h = torch.relu(h @ w2 + b2); logits = h @ w3 + b3
loss = F.cross_entropy(logits, y) + l2 * sum((w ** 2).sum() for w in (w1, w2, w3)); loss.backward()
rel = [((b - a) - (-lr * r.grad)).norm().item() / (lr * r.grad).norm().item() for a, b, r in zip(p0, p1, ref)]
print(json.dumps(rel))
'''
for env in ({}, {"PZ_DW_PAIR": "0"}, {"PZ_GRAD_DTYPE": "fp32"}, {"PZ_DW_PAIR": "0", "PZ_GRAD_DTYPE": "fp32"}):
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    print(env, out.stdout.strip()[-300:], out.stderr.strip()[-300:] if out.returncode else "")
