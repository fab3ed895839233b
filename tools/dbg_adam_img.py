"""Debug: fused clip+Adam+images vs the two-kernel path -- which arena elements differ."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.models.loss import FastSpeech2Loss  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.train.optim import ScheduledOptim  # noqa: E402

DEV = "cuda"
pp, mc, tc = load_named("LJSpeech")
mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 2
b = SyntheticBatches(4, device=DEV, seed=5, phone_counts=[30, 41, 17, 25]).make_batch()
lossf = FastSpeech2Loss(pp, tc)
res = []
for images in (False, True, False):
    torch.manual_seed(3)
    m = FastSpeech2(pp, mc).to(DEV).set_compute_dtype(torch.bfloat16)
    opt = ScheduledOptim(m, tc, mc, 0)
    m.train()
    grads = []
    for it in range(int(os.environ.get("STEPS", 1))):
        hip.set_seed(1234567 + it)
        opt.zero_grad()
        lo = lossf(b, m(*b[2:]), m.film_scalars())
        lo[0].backward()
        opt.arena.finalize_grads()
        grads.append(opt.arena.grad.clone())
        opt.step_count += 1
        a = opt.arena
        fresh = hip.clip_adam_step(a.data, a.grad, opt.exp_avg, opt.exp_avg_sq, 1e-2, opt.betas, opt.eps,
                                   opt.weight_decay, opt.step_count, 1.0, opt.last_grad_norm, opt.skipped_steps,
                                   images=images)
        hip.bump_weight_generation()
        hip.stamp_images(fresh)
    torch.cuda.synchronize()
    names = {}
    for n_, p_ in m.named_parameters():
        names[p_.data_ptr()] = n_
    offs = [(o, a.params[i].numel(), names.get(a.params[i].data_ptr(), "?")) for i, o in enumerate(a.offsets)]
    plan = hip._adam_plan.get((a.data.data_ptr(), a.data.numel())) if images else None
    res.append((a.data.clone(), grads, offs, plan, opt.exp_avg.clone(), opt.exp_avg_sq.clone()))
    del m, opt
(p0, g0, offs, _, m0, v0), (p1, g1, _, plan, m1, v1), (p2, g2, _, _, m2, v2) = res
print('m equal', torch.equal(m0, m1), 'v equal', torch.equal(v0, v1), 'm02', torch.equal(m0, m2), 'ndiff m', int((m0 != m1).sum()), 'ndiff v', int((v0 != v1).sum()))
dm = (m0 != m1).nonzero().flatten()[:5].tolist(); print('m diffs', dm, [(m0[i].item(), m1[i].item()) for i in dm])
print("grad equal run0/run2:", all(torch.equal(x, y) for x, y in zip(g0, g2)), " run0/run1:",
      all(torch.equal(x, y) for x, y in zip(g0, g1)))
print("param equal run0/run2:", torch.equal(p0, p2), " run0/run1:", torch.equal(p0, p1))
d = (p0 != p1).nonzero().flatten().tolist()
print("n diff", len(d))
seen = set()
for i in d:
    for o, k, nm in offs:
        if o <= i < o + k and nm not in seen:
            seen.add(nm)
            print("diff in", nm, "offset", o, "numel", k, "first idx", i)
print("plan ntiles", plan["ntiles"], "nr", plan["nr"], "rtotal", plan["rtotal"], "numel", p0.numel())
print("rest ranges", list(zip(plan["rstart"].tolist()[:10], plan["rcum"].tolist()[:11])))
