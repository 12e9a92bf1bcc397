import os, runpy, sys
sys.path.insert(0, os.getcwd())
if os.environ.get("NO_HASH_PARENT"):
    from uptune_amd.engine import BatchEngine
    BatchEngine.hash_parent = None
sys.argv = ["scripts/c5_bandit.py"] + sys.argv[1:]
runpy.run_path("scripts/c5_bandit.py", run_name="__main__")
