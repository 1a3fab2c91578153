/*
 * TEST INFRASTRUCTURE ONLY -- config 1 (BASELINE.json configs[0]) on the
 * reference's own callers.
 *
 * An echo pair modelled on examples/ws_server/main.c:32-80,131-157 and
 * examples/ws_client/main.c:107-167 (and, for WebSocket over HTTP/2, on
 * test/test_http/test_ws_http2_client_thread.c:24-32,120-150,180-220 and
 * test_http_server_http2_connection.c:7-88,220-230,285-310), built against
 * coldforce's headers and linked with the reference's src/core, src/net,
 * src/http, src/http2, src/ws and src/ws_http2 compiled in place with TLS off
 * (CO_NO_TLS, src/tls_option.cmake:1-11). oracle/Makefile links it twice:
 *
 *   _ref/ws_echo_stock  with the reference's own co_ws_frame.c + co_ws_config.c
 *   _ref/ws_echo_cfws   with libcfws.so in their place (the drop-in)
 *
 * so every frame goes through the reference's unchanged callers:
 *   send    co_ws_send_text -> co_ws_send (co_ws_client.c:427-481)
 *           co_http2_stream_send_ws_text -> co_http2_stream_send_ws_frame
 *           (co_ws_http2_extension.c:166-199) -> co_http2_stream_send_data
 *   receive co_ws_client_on_tcp_receive_ready (co_ws_client.c:178-274),
 *           co_ws_server_on_tcp_receive_ready (co_ws_server.c:85-173), whose
 *           INVALID_FRAME -> HTTP fallback (co_ws_client.c:243-269,
 *           co_ws_server.c:150-168) carries the upgrade request and response;
 *           co_http2_stream_receive_ws_frame (co_ws_http2_extension.c:134-164)
 *
 * Usage:
 *   ws_echo ws-server <port>
 *   ws_echo ws-client ws://127.0.0.1:<port>/ <frames> <payload> <window> <seed>
 *   ws_echo h2-server <port>
 *   ws_echo h2-client http://127.0.0.1:<port>/ <frames> <payload> <window> <seed>
 *
 * The client calls srandom(seed) in on_create (after co_net_setup's
 * srandom(time(NULL)), co_net.c:46), so the upgrade key and every mask key
 * come from that stream. It sends `window` TEXT frames of `payload` bytes
 * (byte j of frame k is 'a' + (j + k) % 26), then one more per echo,
 * checks every echo, and prints one JSON line. The servers echo
 * TEXT/BINARY/CONTINUATION unmasked and stop when the peer closes.
 * CFWS_ECHO_CAPTURE=<path> appends every byte the process sends (send(2),
 * wrapped at link time with --wrap=send) to <path>.
 */
#include <coldforce.h>

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* wire capture: every send(2) of the reference's socket layer lands here    */
/* (co_socket_handle.c:153-170)                                              */
/* ------------------------------------------------------------------------ */
ssize_t __real_send(int fd, const void* buf, size_t len, int flags);

static FILE* g_capture;

ssize_t __wrap_send(int fd, const void* buf, size_t len, int flags)
{
    ssize_t r = __real_send(fd, buf, len, flags);
    if (g_capture != NULL && r > 0)
        fwrite(buf, 1, (size_t)r, g_capture);
    return r;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------------ */
/* app object                                                                */
/* ------------------------------------------------------------------------ */
typedef struct
{
    co_app_t base_app;

    int mode;                      /* 0 ws-server 1 ws-client 2 h2-server 3 h2-client */
    co_tcp_server_t* tcp_server;
    co_list_t* clients;

    co_url_st* url;
    co_ws_client_t* ws_client;
    co_http2_client_t* h2_client;
    co_http2_stream_t* h2_stream;

    unsigned long frames;
    size_t payload;
    unsigned long window;
    unsigned int seed;

    char* text;                    /* payload + NUL, refilled per frame */
    unsigned long sent;
    unsigned long received;
    unsigned long bad;
    unsigned long echoed;          /* server side */
    int upgrade_ok;
    unsigned long warm;            /* echoes before the steady-state clock starts */
    double t0, t1, tw;
    int done;
} app_st;

static void fill_frame(app_st* self, unsigned long k)
{
    for (size_t j = 0; j < self->payload; ++j)
        self->text[j] = (char)('a' + (int)((j + k) % 26));
    self->text[self->payload] = '\0';
}

static int check_frame(const app_st* self, unsigned long k, bool fin, uint8_t opcode, const uint8_t* data,
                       size_t n)
{
    if (!fin || opcode != CO_WS_OPCODE_TEXT || n != self->payload) return 0;
    for (size_t j = 0; j < n; ++j)
        if (data[j] != (uint8_t)('a' + (int)((j + k) % 26))) return 0;
    return 1;
}

static void report(app_st* self)
{
    const double s = self->t1 - self->t0;
    /* steady state: after the first `warm` echoes (the drop-in initialises
       the HIP runtime on its first masked frame, inside the timed span) */
    const double sw = self->t1 - self->tw;
    const unsigned long nw = self->received - self->warm;
    printf("{\"role\": \"client\", \"mode\": \"%s\", \"frames\": %lu, \"payload\": %zu, \"window\": %lu, "
           "\"seed\": %u, \"received\": %lu, \"bad_echo\": %lu, \"upgrade_ok\": %d, \"seconds\": %.6f, "
           "\"frames_per_s\": %.1f, \"us_per_frame\": %.3f, \"warm\": %lu, \"steady_frames_per_s\": %.1f, "
           "\"steady_us_per_frame\": %.3f}\n",
           self->mode == 1 ? "ws" : "h2", self->frames, self->payload, self->window, self->seed, self->received,
           self->bad, self->upgrade_ok, s, s > 0 ? (double)self->received / s : 0.0,
           self->received ? 1e6 * s / (double)self->received : 0.0, self->warm,
           sw > 0 ? (double)nw / sw : 0.0, nw ? 1e6 * sw / (double)nw : 0.0);
    fflush(stdout);
}

static bool send_next(app_st* self)
{
    fill_frame(self, self->sent);
    bool ok;
    if (self->mode == 1)
        ok = co_ws_send_text(self->ws_client, self->text);                 /* co_ws_client.c:473-481 */
    else
        ok = co_http2_stream_send_ws_text(self->h2_stream, true, self->text); /* co_ws_http2_extension.c */
    if (ok) ++self->sent;
    return ok;
}

static void start_sending(app_st* self)
{
    self->upgrade_ok = 1;
    self->t0 = now_s();
    while (self->sent < self->frames && self->sent < self->window)
        if (!send_next(self)) break;
}

static void on_echo(app_st* self, bool fin, uint8_t opcode, const uint8_t* data, size_t n)
{
    if (!check_frame(self, self->received, fin, opcode, data, n)) ++self->bad;
    ++self->received;
    if (self->received == self->warm) self->tw = now_s();
    if (self->sent < self->frames) send_next(self);
    if (self->received == self->frames && !self->done) {
        self->done = 1;
        self->t1 = now_s();
        report(self);
        co_app_stop();
    }
}

/* ------------------------------------------------------------------------ */
/* WebSocket over HTTP/1.1 upgrade (config 1)                                */
/* ------------------------------------------------------------------------ */
static void ws_server_on_receive_frame(app_st* self, co_ws_client_t* ws_client, const co_ws_frame_t* frame,
                                       int error_code)
{
    if (error_code != 0) {
        fprintf(stderr, "ws-server: receive error %d\n", error_code);
        co_list_remove(self->clients, ws_client);
        co_app_stop();
        return;
    }
    const uint8_t opcode = co_ws_frame_get_opcode(frame);
    switch (opcode) {
    case CO_WS_OPCODE_TEXT:
    case CO_WS_OPCODE_BINARY:
    case CO_WS_OPCODE_CONTINUATION:
        co_ws_send(ws_client, co_ws_frame_get_fin(frame), opcode, co_ws_frame_get_payload_data(frame),
                   (size_t)co_ws_frame_get_payload_size(frame));
        ++self->echoed;
        break;
    default:
        co_ws_default_handler(ws_client, frame);
        break;
    }
}

static void ws_server_on_close(app_st* self, co_ws_client_t* ws_client)
{
    co_list_remove(self->clients, ws_client);
    co_app_stop();
}

static void ws_server_on_upgrade(app_st* self, co_ws_client_t* ws_client, const co_http_request_t* request,
                                 int error_code)
{
    if (error_code != 0) {
        fprintf(stderr, "ws-server: bad upgrade request %d\n", error_code);
        co_list_remove(self->clients, ws_client);
        co_app_stop();
        return;
    }
    co_http_response_t* response = co_http_response_create_ws_upgrade(request, NULL, NULL);
    co_http_connection_send_response((co_http_connection_t*)ws_client, response);
    co_http_response_destroy(response);
}

static void ws_server_on_accept(app_st* self, co_tcp_server_t* tcp_server, co_tcp_client_t* tcp_client)
{
    (void)tcp_server;
    co_tcp_accept((co_thread_t*)self, tcp_client);
    co_ws_client_t* ws_client = co_tcp_upgrade_to_ws(tcp_client, NULL);
    co_ws_callbacks_st* cb = co_ws_get_callbacks(ws_client);
    cb->on_upgrade = (co_ws_upgrade_fn)ws_server_on_upgrade;
    cb->on_receive_frame = (co_ws_receive_frame_fn)ws_server_on_receive_frame;
    cb->on_close = (co_ws_close_fn)ws_server_on_close;
    co_list_add_tail(self->clients, ws_client);
}

static void ws_client_on_receive_frame(app_st* self, co_ws_client_t* ws_client, const co_ws_frame_t* frame,
                                       int error_code)
{
    (void)ws_client;
    if (error_code != 0) {
        fprintf(stderr, "ws-client: receive error %d\n", error_code);
        ++self->bad;
        co_app_stop();
        return;
    }
    const uint8_t opcode = co_ws_frame_get_opcode(frame);
    if (opcode == CO_WS_OPCODE_TEXT || opcode == CO_WS_OPCODE_BINARY || opcode == CO_WS_OPCODE_CONTINUATION) {
        on_echo(self, co_ws_frame_get_fin(frame), opcode, co_ws_frame_get_payload_data(frame),
                (size_t)co_ws_frame_get_payload_size(frame));
    } else {
        co_ws_default_handler(ws_client, frame);
    }
}

static void ws_client_on_close(app_st* self, co_ws_client_t* ws_client)
{
    (void)ws_client;
    if (!self->done) fprintf(stderr, "ws-client: closed early after %lu echoes\n", self->received);
    co_app_stop();
}

static void ws_client_on_upgrade(app_st* self, co_ws_client_t* ws_client, const co_http_response_t* response,
                                 int error_code)
{
    (void)ws_client;
    (void)response;
    if (error_code != 0) {
        fprintf(stderr, "ws-client: upgrade failed %d\n", error_code);
        co_app_stop();
        return;
    }
    start_sending(self);
}

static void ws_client_on_connect(app_st* self, co_ws_client_t* ws_client, int error_code)
{
    (void)ws_client;
    if (error_code != 0) {
        fprintf(stderr, "ws-client: connect failed %d\n", error_code);
        co_app_stop();
        return;
    }
    co_http_request_t* request = co_http_request_create_ws_upgrade(self->url->path_and_query, NULL, NULL);
    co_ws_send_upgrade_request(self->ws_client, request);
}

/* ------------------------------------------------------------------------ */
/* WebSocket over HTTP/2 (config 5's callers), cleartext prior knowledge     */
/* ------------------------------------------------------------------------ */
static void h2_server_on_receive_finish(app_st* self, co_http2_client_t* h2, co_http2_stream_t* stream,
                                        const co_http2_header_t* header, const co_http2_data_st* data,
                                        int error_code)
{
    (void)h2;
    if (error_code != 0) {
        fprintf(stderr, "h2-server: receive error %d\n", error_code);
        co_app_stop();
        return;
    }
    const char* protocol = co_http2_stream_get_protocol_mode(stream);
    if (protocol != NULL && strcmp(protocol, "websocket") == 0) {
        co_ws_frame_t* frame = co_http2_stream_receive_ws_frame(stream, data);
        if (frame == NULL) return;
        const uint8_t opcode = co_ws_frame_get_opcode(frame);
        if (opcode == CO_WS_OPCODE_TEXT || opcode == CO_WS_OPCODE_BINARY || opcode == CO_WS_OPCODE_CONTINUATION) {
            co_http2_stream_send_ws_frame(stream, co_ws_frame_get_fin(frame), opcode,
                                          co_ws_frame_get_payload_data(frame),
                                          (size_t)co_ws_frame_get_payload_size(frame));
            ++self->echoed;
        } else {
            co_http2_stream_ws_default_handler(stream, frame);
        }
        co_ws_frame_destroy(frame);
        return;
    }
    if (co_http2_header_validate_ws_connect_request(stream, header)) {
        co_http2_header_t* response = co_http2_header_create_ws_connect_response(NULL, NULL);
        co_http2_stream_send_header(stream, true, response);
        co_http2_stream_set_protocol_mode(stream, "websocket");
    } else {
        fprintf(stderr, "h2-server: not a websocket CONNECT\n");
        co_http2_header_t* response = co_http2_header_create_response(400);
        co_http2_stream_send_header(stream, true, response);
    }
}

static void h2_server_on_close(app_st* self, co_http2_client_t* h2, int error_code)
{
    (void)error_code;
    co_list_remove(self->clients, h2);
    co_app_stop();
}

static void h2_server_on_accept(app_st* self, co_tcp_server_t* tcp_server, co_tcp_client_t* tcp_client)
{
    (void)tcp_server;
    co_tcp_accept((co_thread_t*)self, tcp_client);
    co_http2_client_t* h2 = co_tcp_upgrade_to_http2(tcp_client, NULL);
    co_http2_callbacks_st* cb = co_http2_get_callbacks(h2);
    cb->on_receive_finish = (co_http2_receive_finish_fn)h2_server_on_receive_finish;
    cb->on_close = (co_http2_close_fn)h2_server_on_close;
    co_http2_setting_param_st params[3];
    params[0].id = CO_HTTP2_SETTING_ID_INITIAL_WINDOW_SIZE;
    params[0].value = CO_HTTP2_SETTING_MAX_WINDOW_SIZE;
    params[1].id = CO_HTTP2_SETTING_ID_MAX_CONCURRENT_STREAMS;
    params[1].value = 200;
    params[2].id = CO_HTTP2_SETTING_ID_ENABLE_CONNECT_PROTOCOL;
    params[2].value = 1;
    co_http2_init_settings(h2, params, 3);
    co_list_add_tail(self->clients, h2);
}

static void h2_client_on_receive_finish(app_st* self, co_http2_client_t* h2, co_http2_stream_t* stream,
                                        const co_http2_header_t* header, const co_http2_data_st* data,
                                        int error_code)
{
    (void)h2;
    if (error_code != 0) {
        fprintf(stderr, "h2-client: receive error %d\n", error_code);
        ++self->bad;
        co_app_stop();
        return;
    }
    if (co_http2_stream_get_protocol_mode(stream) == NULL) {
        if (!co_http2_header_validate_ws_connect_response(header)) {
            fprintf(stderr, "h2-client: CONNECT refused\n");
            co_app_stop();
            return;
        }
        co_http2_stream_set_protocol_mode(stream, "websocket");
        start_sending(self);
        return;
    }
    co_ws_frame_t* frame = co_http2_stream_receive_ws_frame(stream, data);
    if (frame == NULL) {
        fprintf(stderr, "h2-client: undecodable ws frame\n");
        ++self->bad;
        return;
    }
    const uint8_t opcode = co_ws_frame_get_opcode(frame);
    if (opcode == CO_WS_OPCODE_TEXT || opcode == CO_WS_OPCODE_BINARY || opcode == CO_WS_OPCODE_CONTINUATION)
        on_echo(self, co_ws_frame_get_fin(frame), opcode, co_ws_frame_get_payload_data(frame),
                (size_t)co_ws_frame_get_payload_size(frame));
    else
        co_http2_stream_ws_default_handler(stream, frame);
    co_ws_frame_destroy(frame);
}

static void h2_client_on_close(app_st* self, co_http2_client_t* h2, int error_code)
{
    (void)h2;
    if (!self->done) fprintf(stderr, "h2-client: closed early (%d) after %lu echoes\n", error_code, self->received);
    co_app_stop();
}

static void h2_client_on_connect(app_st* self, co_http2_client_t* h2, int error_code)
{
    if (error_code != 0) {
        fprintf(stderr, "h2-client: connect failed %d\n", error_code);
        co_app_stop();
        return;
    }
    co_http2_header_t* header = co_http2_header_create_ws_connect_request(self->url->path_and_query, NULL, NULL);
    self->h2_stream = co_http2_create_stream(h2);
    co_http2_stream_send_header(self->h2_stream, true, header);
}

/* ------------------------------------------------------------------------ */
/* app                                                                       */
/* ------------------------------------------------------------------------ */
static bool start_server(app_st* self, uint16_t port)
{
    co_list_ctx_st list_ctx = { 0 };
    list_ctx.destroy_value = self->mode == 0 ? (co_item_destroy_fn)co_ws_client_destroy
                                             : (co_item_destroy_fn)co_http2_client_destroy;
    self->clients = co_list_create(&list_ctx);

    co_net_addr_t local = { 0 };
    co_net_addr_set_family(&local, CO_NET_ADDR_FAMILY_IPV4);
    co_net_addr_set_port(&local, port);
    self->tcp_server = co_tcp_server_create(&local);
    if (self->tcp_server == NULL) return false;
    co_socket_option_set_reuse_addr(co_tcp_server_get_socket(self->tcp_server), true);
    co_tcp_server_callbacks_st* cb = co_tcp_server_get_callbacks(self->tcp_server);
    cb->on_accept = self->mode == 0 ? (co_tcp_accept_fn)ws_server_on_accept : (co_tcp_accept_fn)h2_server_on_accept;
    if (!co_tcp_server_start(self->tcp_server, SOMAXCONN)) return false;
    printf("{\"role\": \"server\", \"listening\": %u}\n", port);
    fflush(stdout);
    return true;
}

static bool app_on_create(app_st* self)
{
    const co_args_st* args = co_app_get_args((co_app_t*)self);
    if (args->count < 3) {
        fprintf(stderr, "usage: ws_echo {ws,h2}-server <port> | {ws,h2}-client <url> <frames> <payload> "
                        "<window> <seed>\n");
        return false;
    }
    const char* m = args->values[1];
    if (strcmp(m, "ws-server") == 0) self->mode = 0;
    else if (strcmp(m, "ws-client") == 0) self->mode = 1;
    else if (strcmp(m, "h2-server") == 0) self->mode = 2;
    else if (strcmp(m, "h2-client") == 0) self->mode = 3;
    else return false;

    const char* cap = getenv("CFWS_ECHO_CAPTURE");
    if (cap != NULL && cap[0] != '\0') {
        g_capture = fopen(cap, "wb");
        if (g_capture == NULL) {
            fprintf(stderr, "cannot open %s: %s\n", cap, strerror(errno));
            return false;
        }
    }

    if (self->mode == 0 || self->mode == 2) return start_server(self, (uint16_t)atoi(args->values[2]));

    if (args->count < 7) return false;
    self->url = co_url_create(args->values[2]);
    self->frames = strtoul(args->values[3], NULL, 10);
    self->payload = (size_t)strtoull(args->values[4], NULL, 10);
    self->window = strtoul(args->values[5], NULL, 10);
    self->seed = (unsigned)strtoul(args->values[6], NULL, 10);
    if (self->window == 0) self->window = 1;
    self->warm = self->frames >= 10000 ? 1000 : self->frames / 10;
    if (self->warm == 0) self->warm = 1;
    self->text = (char*)malloc(self->payload + 1);
    if (self->text == NULL || self->frames == 0) return false;

    /* after co_net_setup's srandom(time(NULL)) (co_net.c:46): the upgrade
       key and every mask key come from this stream */
    srandom(self->seed);

    co_net_addr_t local = { 0 };
    co_net_addr_set_family(&local, CO_NET_ADDR_FAMILY_IPV4);
    co_tls_ctx_st tls_ctx = { 0 };
    if (self->mode == 1) {
        self->ws_client = co_ws_client_create(self->url->origin, &local, &tls_ctx);
        if (self->ws_client == NULL) return false;
        co_ws_callbacks_st* cb = co_ws_get_callbacks(self->ws_client);
        cb->on_connect = (co_ws_connect_fn)ws_client_on_connect;
        cb->on_upgrade = (co_ws_upgrade_fn)ws_client_on_upgrade;
        cb->on_receive_frame = (co_ws_receive_frame_fn)ws_client_on_receive_frame;
        cb->on_close = (co_ws_close_fn)ws_client_on_close;
        return co_ws_start_connect(self->ws_client);
    }
    self->h2_client = co_http2_client_create(self->url->origin, &local, &tls_ctx);
    if (self->h2_client == NULL) return false;
    co_http2_setting_param_st params[2];
    params[0].id = CO_HTTP2_SETTING_ID_INITIAL_WINDOW_SIZE;
    params[0].value = CO_HTTP2_SETTING_MAX_WINDOW_SIZE;
    params[1].id = CO_HTTP2_SETTING_ID_ENABLE_CONNECT_PROTOCOL;
    params[1].value = 1;
    co_http2_init_settings(self->h2_client, params, 2);
    co_http2_callbacks_st* cb = co_http2_get_callbacks(self->h2_client);
    cb->on_connect = (co_http2_connect_fn)h2_client_on_connect;
    cb->on_receive_finish = (co_http2_receive_finish_fn)h2_client_on_receive_finish;
    cb->on_close = (co_http2_close_fn)h2_client_on_close;
    return co_http2_start_connect(self->h2_client);
}

static void app_on_destroy(app_st* self)
{
    if (self->mode == 1 && self->ws_client != NULL) co_ws_client_destroy(self->ws_client);
    if (self->mode == 3 && self->h2_client != NULL) co_http2_client_destroy(self->h2_client);
    if (self->tcp_server != NULL) co_tcp_server_destroy(self->tcp_server);
    if (self->clients != NULL) co_list_destroy(self->clients);
    if (self->url != NULL) co_url_destroy(self->url);
    if (self->mode == 0 || self->mode == 2) {
        printf("{\"role\": \"server\", \"echoed\": %lu}\n", self->echoed);
        fflush(stdout);
    }
    free(self->text);
    if (g_capture != NULL) fclose(g_capture);
    g_capture = NULL;
}

int main(int argc, char* argv[])
{
    app_st self;
    memset(&self, 0, sizeof self);
    int rc = co_net_app_start((co_app_t*)&self, "ws-echo", (co_app_create_fn)app_on_create,
                              (co_app_destroy_fn)app_on_destroy, argc, argv);
    if (self.mode == 1 || self.mode == 3) {
        if (!self.done) return 3;
        if (self.bad != 0) return 4;
    }
    return rc;
}
