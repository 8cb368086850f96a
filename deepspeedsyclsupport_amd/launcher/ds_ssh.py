"""`ds_ssh`: run one shell command on every host of a hostfile (reference `bin/ds_ssh`, a pdsh wrapper).

Uses pdsh when it is installed (same fan-out as the reference); otherwise starts one `ssh` per host in parallel
and prefixes each output line with its host. Exit status: the first non-zero host status, else 0.
"""
import argparse
import shutil
import subprocess
import sys
import threading

from .runner import DEFAULT_HOSTFILE, fetch_hostfile


def main(argv=None):
    p = argparse.ArgumentParser(prog="ds_ssh")
    p.add_argument("-f", "--hostfile", default=DEFAULT_HOSTFILE)
    p.add_argument("command", nargs=argparse.REMAINDER)
    args = p.parse_args(argv)
    hosts = list((fetch_hostfile(args.hostfile) or {}).keys())
    if not hosts:
        print(f"ds_ssh: no hosts in {args.hostfile}", file=sys.stderr)
        return 1
    cmd = " ".join(args.command)
    if shutil.which("pdsh"):
        return subprocess.call(["pdsh", "-S", "-w", ",".join(hosts), cmd])
    status = {}

    def one(h):
        proc = subprocess.Popen(["ssh", "-o", "BatchMode=yes", h, cmd], stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, text=True)
        for line in proc.stdout:
            sys.stdout.write(f"{h}: {line}")
        status[h] = proc.wait()

    threads = [threading.Thread(target=one, args=(h, )) for h in hosts]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return next((status[h] for h in hosts if status.get(h)), 0)
