"""Duplicate-classification probe: the single-GPU path and 2 host-transport ranks."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"), os.path.join(os.path.dirname(__file__), "..", "oracle"),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
import numpy as np
import oracle as O
import s3imph
import torch
def main():
  keys = [b"x/%05d/" % i for i in range(3000)]
  keys[2500] = keys[10]
  blob, offs = O.keys_to_blob(keys)
  print("oracle fnv of dup key %016x" % O.lib().fnv1a64(keys[10]))
  try:
      s3imph.build_host(blob, offs)
  except s3imph.MPHFError as e:
      print("single:", e.status, e)
  os.environ["S3IMPH_DEBUG"] = "1"
  import test_gpu_dist as T
  res = T._run(2, T._shards(blob, offs, [0, 1500, 3000]), 3000, 1 << 20, "route")
  print(res)


if __name__ == "__main__":
  main()
