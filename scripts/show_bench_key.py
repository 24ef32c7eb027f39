"""Prints one key of the last bench JSON line in a log: show_bench_key.py LOG KEY"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)[sys.argv[2]]
print({k: v for k, v in d.items() if not isinstance(v, (dict, list)) or k.endswith("log")})
