"""One-screen summary of a bench.py JSON line (main window, steady state, side windows)."""
import json
import sys

ln = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(ln)
c = d.get("config", {})
print("main %.2fM env-steps/s, %.2f us/step (kernel %.2f us), resets %s, window_ms %s" % (
    d["value"] / 1e6, d["ms_per_step"] * 1e3, c.get("step_kernel_ms", 0) * 1e3, c.get("resets"), c.get("window_ms")))
s = d.get("steady_state")
if s:
    print("steady %.2fM, %.2f us/step (kernel %.2f us), resets %s" % (s["value"] / 1e6, s["ms_per_step"] * 1e3,
                                                                     s["step_kernel_ms"] * 1e3, s["resets"]))
for k in ("side_c3", "side_c5", "side_c4"):
    v = d.get(k)
    if v is None:
        continue
    if "error" in v:
        print(k, "ERROR", v["error"])
        continue
    r = v.get("roofline", {})
    print("%s %.4gM env-steps/s, %.3f ms/step, resets %s, roofline %s %.3f, wall %.1f s" % (
        k, v["value"] / 1e6, v["ms_per_step"], v.get("resets"), r.get("unit"), r.get("frac", 0), v.get("wall_s", 0)))
cb = d.get("cpu_baseline")
if cb:
    print("cpu_baseline %.0f on %d threads (1 thread %.0f)" % (cb["value"], cb["cores"], cb["one_thread"]["value"]))
