import resource, subprocess, sys, time, os
sys.path.insert(0, "tools"); sys.path.insert(0, ".")
env = dict(os.environ, LD_LIBRARY_PATH=os.getcwd() + "/click_amd:/opt/rocm/lib")
for mode in ("cpu", "dropin"):
    for limit in (2000000, 8000000):
        r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t = time.time()
        p = subprocess.run(["click_integration/bin/click-" + mode, "click_integration/conf/c1-forward.click",
                            "LIMIT=%d" % limit, "BURST=32", "-h", "out.rate"], capture_output=True, text=True, env=env,
                           timeout=120)
        w = time.time() - t
        r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        print(mode, limit, "wall %.2f" % w, "user %.2f sys %.2f" % (r1.ru_utime - r0.ru_utime, r1.ru_stime - r0.ru_stime),
              "maxrss_MB %.0f" % (r1.ru_maxrss / 1024), "minflt", r1.ru_minflt - r0.ru_minflt, p.stdout.split()[-1:],
              flush=True)
