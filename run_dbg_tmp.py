import faulthandler, sys
f = open("/tmp/stacks.txt", "w")
faulthandler.dump_traceback_later(40, repeat=True, file=f)
sys.argv = ["xot", "run", "llama-3.2-1b", "--prompt", "Who are you?", "--max-generate-tokens", "8", "--disable-tui"]
from xotorch_support_jetson_amd.main import run
run()
