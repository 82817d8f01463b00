"""DIAGNOSTIC: linear+relu vs torch._addmm_activation at the DQN shapes."""
import torch

x = torch.randn(65536, 198, device="cuda")
lin = torch.nn.Linear(198, 256).cuda()
lin2 = torch.nn.Linear(256, 256).cuda()


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


with torch.no_grad():
    a = lambda: torch.relu(lin2(torch.relu(lin(x))))  # noqa: E731
    b = lambda: torch._addmm_activation(lin2.bias, torch._addmm_activation(lin.bias, x, lin.weight.t()),  # noqa: E731
                                        lin2.weight.t())
    ya, yb = a(), b()
    print("equal", torch.equal(ya, yb), "maxdiff", float((ya - yb).abs().max()))
    print(f"linear+relu {timed(a):.1f} us, addmm_activation {timed(b):.1f} us")
