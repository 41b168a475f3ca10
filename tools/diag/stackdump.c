/* A SIGUSR2 handler that writes the receiving thread's native backtrace (libc backtrace) and this
 * process's executable mappings to stderr: for a diagnostic that finds a thread spinning inside a
 * library (tools/diag/rss_layout.py sends the signal to the stuck thread).  Resolve the frames with
 * addr2line against the same build of the library, offset = address - mapping start + file offset.
 * Build: gcc -O1 -g -shared -fPIC -o tools/diag/libstackdump.so tools/diag/stackdump.c */
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_signal(int sig) {
  (void)sig;
  void* frames[64];
  const int n = backtrace(frames, 64);
  static const char head[] = "---- native backtrace ----\n";
  (void)!write(2, head, sizeof head - 1);
  backtrace_symbols_fd(frames, n, 2);
  static const char maps[] = "---- maps (r-x) ----\n";
  (void)!write(2, maps, sizeof maps - 1);
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  char buf[8192], line[1024];
  size_t ln = 0;
  ssize_t k;
  while ((k = read(fd, buf, sizeof buf)) > 0) {
    for (ssize_t i = 0; i < k; ++i) {
      if (ln < sizeof line - 1) line[ln++] = buf[i];
      if (buf[i] == '\n') {
        if (ln > 30 && memchr(line, 'x', 40) && memchr(line, '/', ln)) (void)!write(2, line, ln);
        ln = 0;
      }
    }
  }
  close(fd);
}

int stackdump_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sa.sa_flags = SA_RESTART;
  sigemptyset(&sa.sa_mask);
  void* warm[2];
  backtrace(warm, 2);  /* loads libgcc_s now, not inside the handler */
  return sigaction(SIGUSR2, &sa, 0);
}
