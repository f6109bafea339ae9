// rt_queue.cpp — the render queue: the WorkerPool[WorkMsg, ResponseMsg] that
// raytracer.nim and gui.nim drive (src/concurrency/workerpool.nim,
// src/raytracer.nim:13-38, src/gui.nim:98-122,206-280), over the GPU.
//
// The reference runs renderLine on N CPU threads, one queued line per
// message. Here one host thread per queue drains the work queue in batches:
// the longest run of queued lines that share options, framebuffer, step and
// maxStep and follow each other at `step` becomes ONE rt_render_lines call
// (one kernel launch over the whole run), so the GUI's "queue every line of
// this refinement level" pattern costs a launch per level, not per line.
// Every message still gets its own response, in queue order; a batch's Stats
// ride on its last line's response and the others carry zero Stats (the
// callers only sum them: raytracer.nim:95, gui.nim:261). State machine, return
// values and reset semantics follow workerpool.nim; commands complete before
// they return, so the queue is always "ready".
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "../../include/rtmi.h"
#include "rt_common.h"

namespace {

struct Work {
  rt_options opts;
  float* fb;
  int32_t fb_w, fb_h, line, step, max_step;
};

bool same_batch(const Work& a, const Work& b) {
  return a.fb == b.fb && a.fb_w == b.fb_w && a.fb_h == b.fb_h && a.step == b.step && a.max_step == b.max_step &&
         std::memcmp(&a.opts, &b.opts, sizeof a.opts) == 0 && b.line == a.line + a.step;
}

// renderLine's defaults for a zero step / maxStep (raytracer.nim:26-27)
int32_t or_one(int32_t v) { return v == 0 ? 1 : v; }

}  // namespace

struct rt_queue {
  rt_scene* scene = nullptr;
  std::mutex mu;
  std::condition_variable cv;       // worker: work or a command arrived
  std::condition_variable idle_cv;  // callers: the in-flight batch finished
  std::deque<Work> work;
  std::deque<rt_response> results;
  int state = RT_QUEUE_STOPPED;
  bool busy = false;
  bool quit = false;
  std::thread worker;

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return quit || (state == RT_QUEUE_RUNNING && !work.empty()); });
      if (quit) return;
      // the longest contiguous run of compatible lines at the queue head
      std::deque<Work> batch;
      batch.push_back(work.front());
      work.pop_front();
      while (!work.empty() && same_batch(batch.back(), work.front())) {
        batch.push_back(work.front());
        work.pop_front();
      }
      busy = true;
      lk.unlock();
      const Work& w0 = batch.front();
      rt_stats st{};
      const int rc = rt_render_lines(scene, &w0.opts, w0.fb, w0.fb_w, w0.fb_h, w0.line,
                                     batch.back().line + 1, w0.step, w0.max_step, &st);
      const std::string err = rc ? std::string(rt_last_error()) : std::string();
      lk.lock();
      for (size_t i = 0; i < batch.size(); ++i) {
        rt_response r{};
        r.line = batch[i].line;
        r.status = rc;
        if (i + 1 == batch.size()) r.stats = st;
        if (rc) std::strncpy(r.error, err.c_str(), sizeof r.error - 1);
        results.push_back(r);
      }
      busy = false;
      idle_cv.notify_all();
    }
  }

  // waits for the in-flight batch (stop / reset / shutdown return "ready")
  void wait_idle(std::unique_lock<std::mutex>& lk) {
    idle_cv.wait(lk, [&] { return !busy; });
  }
};

extern "C" {

int rt_queue_create(rt_scene* scene, rt_queue** out) {
  if (!scene || !out) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  *out = nullptr;
  rt_queue* q = new rt_queue();
  q->scene = scene;
  try {
    q->worker = std::thread([q] { q->run(); });
  } catch (...) {
    delete q;
    return rtmi_fail_msg(RT_E_NOMEM, "cannot start the queue thread");
  }
  *out = q;
  return RT_OK;
}

// workerpool.nim start: only from the stopped state
int rt_queue_start(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::lock_guard<std::mutex> lk(q->mu);
  if (q->state != RT_QUEUE_STOPPED) return 0;
  q->state = RT_QUEUE_RUNNING;
  q->cv.notify_all();
  return 1;
}

// workerpool.nim stop: only while running; the batch in flight completes
// (its responses are delivered), queued lines stay queued
int rt_queue_stop(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::unique_lock<std::mutex> lk(q->mu);
  if (q->state != RT_QUEUE_RUNNING) return 0;
  q->state = RT_QUEUE_STOPPED;
  q->wait_idle(lk);
  return 1;
}

int rt_queue_state(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::lock_guard<std::mutex> lk(q->mu);
  return q->state;
}

int rt_queue_is_ready(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  return 1;
}

int rt_queue_work(rt_queue* q, const rt_options* opts, float* fb, int32_t fb_w, int32_t fb_h, int32_t line,
                  int32_t step, int32_t max_step) {
  if (!q || !opts || !fb) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  if (fb_w != opts->width || fb_h != opts->height)
    return rtmi_fail_msg(RT_E_INVALID, "framebuffer size does not match the options");
  if (line < 0 || line >= fb_h) return rtmi_fail_msg(RT_E_INVALID, "line out of range");
  std::lock_guard<std::mutex> lk(q->mu);
  if (q->state == RT_QUEUE_SHUTDOWN) return rtmi_fail_msg(RT_E_INVALID, "queue is shut down");
  q->work.push_back(Work{*opts, fb, fb_w, fb_h, line, or_one(step), or_one(max_step)});
  q->cv.notify_all();
  return RT_OK;
}

int rt_queue_try_recv(rt_queue* q, rt_response* out) {
  if (!q || !out) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(q->mu);
  if (q->results.empty()) return 0;
  *out = q->results.front();
  q->results.pop_front();
  if (out->status) rtmi_fail_msg(out->status, out->error);
  return 1;
}

int rt_queue_pending(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::lock_guard<std::mutex> lk(q->mu);
  return (int)(q->work.size() + (q->busy ? 1 : 0));
}

// workerpool.nim reset: stop if running, then drop queued work and
// undelivered responses; the queue is left stopped
int rt_queue_reset(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::unique_lock<std::mutex> lk(q->mu);
  if (q->state == RT_QUEUE_SHUTDOWN) return 0;
  q->state = RT_QUEUE_STOPPED;
  q->wait_idle(lk);
  q->work.clear();
  q->results.clear();
  return 1;
}

// workerpool.nim shutdown: no more work is accepted or started
int rt_queue_shutdown(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  std::unique_lock<std::mutex> lk(q->mu);
  if (q->state == RT_QUEUE_SHUTDOWN) return 0;
  q->state = RT_QUEUE_SHUTDOWN;
  q->wait_idle(lk);
  return 1;
}

// workerpool.nim close (after shutdown) + free; destroys a queue in any state
int rt_queue_destroy(rt_queue* q) {
  if (!q) return rtmi_fail_msg(RT_E_INVALID, "null queue");
  {
    std::unique_lock<std::mutex> lk(q->mu);
    q->state = RT_QUEUE_SHUTDOWN;
    q->quit = true;
    q->cv.notify_all();
  }
  if (q->worker.joinable()) q->worker.join();
  delete q;
  return RT_OK;
}

}  // extern "C"
