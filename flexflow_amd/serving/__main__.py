"""python -m flexflow_amd.serving --model-repository DIR [--http-port P] [--host H] [FFConfig flags]"""
import argparse
import sys

from .server import InferenceServer


def main(argv=None):
    ap = argparse.ArgumentParser(prog="flexflow_amd.serving")
    ap.add_argument("--model-repository", required=True)
    ap.add_argument("--http-port", type=int, default=8000)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--strict", action="store_true", help="exit if any model fails to load")
    ap.add_argument("-v", "--verbose", action="store_true")
    args, ff_flags = ap.parse_known_args(argv)
    srv = InferenceServer(args.model_repository, args.host, args.http_port, ff_flags, args.verbose, args.strict)
    errs = srv.repo.load_all(strict=args.strict)
    for n, e in errs.items():
        print(f"[serving] model {n} failed to load: {e}", file=sys.stderr, flush=True)
    srv.httpd.ready.set()
    print(f"[serving] {len(srv.repo.models)} model(s) ready on http://{srv.url}", flush=True)
    try:
        srv.httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
